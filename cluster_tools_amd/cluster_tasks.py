"""Job runtime of the watershed path's tasks: configs, per-job configs and scripts, submission to
a local process pool / Slurm / LSF, log-based success checks and block-level retry.

The on-disk contract is the reference's (cluster_tools/cluster_tasks.py:25-654); the job scripts
and callers rely on it, so it is kept exactly:
* configs: ``config_dir/global.config`` and ``config_dir/<task_name>.config``, taken verbatim when
  present (not merged with the defaults);
* job configs: ``tmp_folder/<task_name>_job_[<prefix>_]<id>.config`` = task config + its
  ``block_list`` (round robin ``block_list[id::n_jobs]``, or consecutive runs);
* job scripts: the task's module copied to ``tmp_folder/<task_name>.py`` with the configured
  shebang as first line, called with the job config path;
* logs: ``tmp_folder/logs/<job>_<id>.log`` (stdout) and ``tmp_folder/error_logs/<job>_<id>.err``;
  success and processed blocks are read from the log lines (utils/parse_utils.py); failed jobs
  are retried with their unprocessed blocks while retries remain, the task allows it and fewer
  than half of the jobs failed — otherwise the task log is renamed ``*_failed.log`` and
  FailedJobsError is raised;
* the luigi target is ``tmp_folder/<task_name>.log``.

GPU placement: a local job process opens one libctws handle on the device ``job_id % n_gpus``
(CTWS_DEVICE in the job environment), so ``max_jobs`` jobs share the node's GPUs.
"""
import json
import os
import shutil
import stat
import subprocess
import time
from concurrent import futures
from datetime import datetime, timedelta
from multiprocessing import cpu_count

from . import luigi_compat as luigi
from .utils.parse_utils import parse_blocks_task, parse_job, parse_job_lsf
from .utils.task_utils import DummyTask

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DEFAULT_GLOBAL_CONFIG = {"block_shape": [50, 512, 512], "shebang": "#! /bin/python", "roi_begin": None,
                         "roi_end": None, "groupname": "kreshuk", "partition": None, "max_num_retries": 0,
                         "block_list_path": None}
DEFAULT_TASK_CONFIG = {'threads_per_job': 1, 'time_limit': 60, 'mem_limit': 1., 'qos': 'normal'}


class FailedJobsError(Exception):
    pass


# ---- GPU placement ---------------------------------------------------------------------------
def _count_gpus():
    """GPUs this process may use: the visibility lists (ROCR_VISIBLE_DEVICES applies first on
    ROCm, then HIP_/CUDA_VISIBLE_DEVICES), else the render nodes of the machine."""
    counts = []
    for var in ('ROCR_VISIBLE_DEVICES', 'HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES'):
        v = os.environ.get(var)
        if v is not None:
            counts.append(len([d for d in v.split(',') if d.strip()]))
    if counts:
        return min(counts)
    try:
        return sum(1 for d in os.listdir('/dev/dri') if d.startswith('renderD'))
    except OSError:
        return 0


def _job_env(job_id=None):
    """Environment of a job process: the package importable; local jobs get a GPU each."""
    env = dict(os.environ)
    paths = [p for p in env.get('PYTHONPATH', '').split(os.pathsep) if p]
    if _PKG_ROOT not in paths:
        env['PYTHONPATH'] = os.pathsep.join([_PKG_ROOT] + paths)
    if job_id is not None and 'CTWS_DEVICE' not in env:
        n = _count_gpus()
        if n:
            env['CTWS_DEVICE'] = str(job_id % n)
    return env


# ---- job partitioning ------------------------------------------------------------------------
def split_blocks(block_list, n_jobs, consecutive=False):
    """Per-job block lists: round robin, or consecutive runs whose sizes differ by at most one
    (the first len % n_jobs jobs get one more)."""
    if not consecutive:
        return [block_list[j::n_jobs] for j in range(n_jobs)]
    q, r = divmod(len(block_list), n_jobs)
    out, start = [], 0
    for j in range(n_jobs):
        n = q + (1 if j < r else 0)
        out.append(list(block_list[start:start + n]))
        start += n
    return out


class _Paths:
    """File layout of a task's jobs under tmp_folder."""

    def __init__(self, tmp_folder, task_name, job_prefix=None):
        self.tmp = tmp_folder
        self.task = task_name
        self.prefix = job_prefix
        self.job = task_name if job_prefix is None else '%s_%s' % (task_name, job_prefix)

    def config(self, job_id):
        mid = '' if self.prefix is None else '%s_' % self.prefix
        return os.path.join(self.tmp, '%s_job_%s%s.config' % (self.task, mid, job_id))

    def log(self, job_id):
        return os.path.join(self.tmp, 'logs', '%s_%i.log' % (self.job, job_id))

    def err(self, job_id):
        return os.path.join(self.tmp, 'error_logs', '%s_%i.err' % (self.job, job_id))

    def log_prefix(self):
        return os.path.join(self.tmp, 'logs', '%s_' % self.job)

    def script(self):
        return os.path.join(self.tmp, self.task + '.py')


# ---- tasks -------------------------------------------------------------------------------------
class BaseClusterTask(luigi.Task):
    """A task that runs as jobs.  Subclasses implement run_impl (global_config_values -> init ->
    get_task_config -> prepare_jobs -> submit_jobs -> wait_for_jobs -> check_jobs); the backend
    classes below implement prepare / submit / wait."""
    tmp_folder = luigi.Parameter()
    max_jobs = luigi.IntParameter()
    config_dir = luigi.Parameter()
    allow_retry = True
    n_retries = 0

    # -- lifecycle
    def run(self):
        self.make_dirs()
        self._write_log("Start task %s" % self.task_name)
        try:
            self.run_impl()
        except FailedJobsError:
            raise
        except Exception as e:
            self._write_log("task failed in `run_impl` with %s" % str(e))
            self._mark_failed()
            raise
        self._write_log("Done task %s" % self.task_name)

    def init(self, shebang):
        self._write_script_file(shebang)

    def output(self):
        return luigi.LocalTarget(os.path.join(self.tmp_folder, self.task_name + '.log'))

    def make_dirs(self):
        for sub in ('', 'logs', 'error_logs'):
            os.makedirs(os.path.join(self.tmp_folder, sub), exist_ok=True)
        self._write_log('created tmp-folder and log dirs @ %s' % self.tmp_folder)

    # -- configs
    def _read_config(self, name, default, what):
        path = os.path.join(self.config_dir, name)
        if os.path.exists(path):
            self._write_log("reading %s config from %s" % (what, path))
            with open(path) as f:
                return json.load(f)
        self._write_log("reading default %s config" % what)
        return default()

    def get_task_config(self):
        return self._read_config(self.task_name + '.config', self.default_task_config, 'task')

    def get_global_config(self):
        return self._read_config('global.config', self.default_global_config, 'global')

    @staticmethod
    def default_task_config():
        return dict(DEFAULT_TASK_CONFIG)

    @staticmethod
    def default_global_config():
        return dict(DEFAULT_GLOBAL_CONFIG)

    def global_config_values(self, with_block_list_path=False):
        gc = self.get_global_config()
        vals = (gc["shebang"], gc["block_shape"], gc.get("roi_begin"), gc.get("roi_end"))
        return vals + (gc.get("block_list_path"),) if with_block_list_path else vals

    def clean_up_for_retry(self, block_list, prefix=None):
        pass

    # -- the blockwise schedule every task of the path shares
    def blocks_to_process(self, shape, block_shape, roi_begin=None, roi_end=None, block_list_path=None,
                          job_prefix=None):
        """First attempt: the blocks of the volume (or of its roi / the given block list).  A
        retry: the blocks no job of the previous attempt processed, after the task's clean-up."""
        if self.n_retries > 0:
            self.clean_up_for_retry(self.block_list, job_prefix)
            return self.block_list
        from cluster_tools_amd.utils.volume_utils import blocks_in_volume
        return blocks_in_volume(shape, block_shape, roi_begin, roi_end, block_list_path=block_list_path)

    def run_jobs(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        """Write the job configs, submit, wait and check (retrying failed blocks per the global
        config); block_list None = one job that gets the config as is."""
        if block_list is not None:
            self._write_log('scheduling %i blocks to be processed' % len(block_list))
        self.prepare_jobs(n_jobs, block_list, config, job_prefix, consecutive_blocks)
        self.submit_jobs(n_jobs, job_prefix)
        self.wait_for_jobs(job_prefix)
        self.check_jobs(n_jobs, job_prefix)

    # -- results and retry
    @staticmethod
    def parse_jobs(log_prefix, max_jobs):
        return [j for j in range(max_jobs) if parse_job(log_prefix + '%i.log' % j, j)]

    def check_jobs(self, n_jobs, job_prefix=None):
        paths = _Paths(self.tmp_folder, self.task_name, job_prefix)
        ok = self.parse_jobs(paths.log_prefix(), n_jobs)
        if len(ok) == n_jobs:
            self._write_log("%s finished successfully" % self.task_name)
            return
        failed = sorted(set(range(n_jobs)) - set(ok))
        self._write_log("%s failed for jobs:" % self.task_name)
        self._write_log("%s" % ', '.join(str(j) for j in failed))
        retries_left = self.n_retries < self.get_global_config().get('max_num_retries', 0)
        if retries_left and self.allow_retry and len(failed) / n_jobs < 0.5:
            todo = self.get_failed_blocks(n_jobs, ok, job_prefix)
            self._write_log("resubmitting %i failed blocks in %i retry attempt" % (len(todo), self.n_retries + 1))
            self.n_retries += 1
            self.block_list = todo
            self.run()
            return
        self._mark_failed()
        raise FailedJobsError("Task: %s failed for %i / %i jobs" % (self.task_name, len(failed), n_jobs))

    def get_failed_blocks(self, n_jobs, passed_jobs=(), job_prefix=None):
        """The scheduled blocks that no job logged as processed (blocks of passed jobs count as
        processed: their job configs list them)."""
        paths = _Paths(self.tmp_folder, self.task_name, job_prefix)
        done = set()
        for j in passed_jobs:
            if os.path.exists(paths.config(j)):
                with open(paths.config(j)) as f:
                    done.update(json.load(f).get('block_list') or [])
        done.update(parse_blocks_task(paths.log_prefix(), n_jobs, passed_jobs))
        return sorted(set(self.block_list) - done)

    # -- job files
    def _write_log(self, msg):
        with open(self.output().path, 'a') as f:
            f.write('%s: %s\n' % (str(datetime.now()), msg))

    def _mark_failed(self):
        src = self.output().path
        dst = src[:-4] + '_failed.log'
        self._write_log("move log from %s to %s" % (src, dst))
        shutil.move(src, dst)

    def _config_path(self, job_id, job_prefix=None):
        return _Paths(self.tmp_folder, self.task_name, job_prefix).config(job_id)

    def _write_job_config(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        paths = _Paths(self.tmp_folder, self.task_name, job_prefix)
        if block_list is None:
            assert n_jobs == 1
            with open(paths.config(0), 'w') as f:
                json.dump(config, f)
        else:
            self.block_list = block_list
            for j, blocks in enumerate(split_blocks(block_list, n_jobs, consecutive_blocks)):
                with open(paths.config(j), 'w') as f:
                    json.dump(dict(config, block_list=blocks), f)
        self._write_log('written config for %i jobs' % n_jobs)

    def _write_script_file(self, shebang):
        assert os.path.exists(self.src_file), self.src_file
        dst = _Paths(self.tmp_folder, self.task_name).script()
        with open(self.src_file) as f:
            body = f.read().split('\n', 1)
        with open(dst, 'w') as f:
            f.write(shebang + '\n' + (body[1] if len(body) > 1 else ''))
        os.chmod(dst, os.stat(dst).st_mode | stat.S_IEXEC)
        self._write_log('copied python script from %s to %s' % (self.src_file, dst))

    # -- backend
    def prepare_jobs(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        self._write_job_config(n_jobs, block_list, config, job_prefix, consecutive_blocks)

    def submit_jobs(self, n_jobs, job_prefix=None):
        raise NotImplementedError

    def wait_for_jobs(self, job_prefix=None):
        raise NotImplementedError


def _poll_until_gone(list_cmd, empty_message, ids, merge_stderr):
    """Poll a scheduler listing every 10 s until none of `ids` is listed any more."""
    while True:
        time.sleep(10)
        try:
            out = subprocess.check_output([list_cmd], shell=True,
                                          stderr=subprocess.STDOUT if merge_stderr else None).decode()
        except subprocess.CalledProcessError as e:
            if e.output.decode().rstrip() == empty_message:
                return
            raise
        live = [int(ln.split()[0]) for ln in out.split('\n') if ln.strip()]
        if not any(i in ids for i in live):
            return


class LocalTask(BaseClusterTask):
    """Jobs as local subprocesses, all started at once (their number is bounded by the cores)."""
    max_local_jobs = cpu_count()

    def _run_job(self, job_id, job_prefix):
        paths = _Paths(self.tmp_folder, self.task_name, job_prefix)
        script, cfg = paths.script(), paths.config(job_id)
        assert os.path.exists(script) and os.path.exists(cfg)
        with open(paths.log(job_id), 'w') as out, open(paths.err(job_id), 'w') as err:
            subprocess.call([script, cfg], stdout=out, stderr=err, env=_job_env(job_id))

    def submit_jobs(self, n_jobs, job_prefix=None):
        assert n_jobs <= self.max_local_jobs, \
            "Trying to submit %i local jobs but limit is %i. Did you forget to set the target to slurm or lsf?" % \
            (n_jobs, self.max_local_jobs)
        # each job is its own OS process; threads only wait for them
        with futures.ThreadPoolExecutor(n_jobs) as pool:
            for r in [pool.submit(self._run_job, j, job_prefix) for j in range(n_jobs)]:
                r.result()

    def wait_for_jobs(self, job_prefix=None):
        pass


class SlurmTask(BaseClusterTask):
    """Jobs submitted with sbatch (one batch script per task, job id as argument), polled with
    squeue."""

    @staticmethod
    def _time(minutes):
        t = timedelta(minutes=minutes)
        h, rem = divmod(t.seconds, 3600)
        return "%i-%i:%i:%i" % (t.days, h, rem // 60, rem % 60)

    @staticmethod
    def _mem(gb):
        return "%iG" % gb if gb > 1 else "%iM" % int(gb * 1000)

    def _batch_script(self, job_prefix=None):
        gc, tc = self.get_global_config(), self.get_task_config()
        paths = _Paths(self.tmp_folder, self.task_name, job_prefix)
        opts = ["-A %s" % gc.get('groupname', 'kreshuk'), "-N 1", "-c %i" % tc.get("threads_per_job", 1),
                "--mem %s" % self._mem(tc.get("mem_limit", 2)), "-t %s" % self._time(tc.get("time_limit", 60)),
                "--qos=%s" % tc.get("qos", "normal")]
        if gc.get('partition') is not None:
            opts.append("-p=%s" % gc['partition'])
        if tc.get('gpus_per_job', 0):
            opts.append("--gres=gpu:%i" % tc['gpus_per_job'])
        body = ["#!/bin/bash"] + ["#SBATCH " + o for o in opts] + ["%s %s" % (paths.script(), paths.config('$1'))]
        path = os.path.join(self.tmp_folder, 'slurm_%s.sh' % paths.job)
        with open(path, 'w') as f:
            f.write("\n".join(body))
        return path

    def prepare_jobs(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        super().prepare_jobs(n_jobs, block_list, config, job_prefix, consecutive_blocks)
        self._batch_script(job_prefix)

    def submit_jobs(self, n_jobs, job_prefix=None):
        paths = _Paths(self.tmp_folder, self.task_name, job_prefix)
        script = os.path.join(self.tmp_folder, 'slurm_%s.sh' % paths.job)
        self.slurm_ids = []
        for j in range(n_jobs):
            cmd = ['sbatch', '-o', paths.log(j), '-e', paths.err(j), '-J', '%s_%i' % (paths.job, j), script, str(j)]
            out = subprocess.check_output(cmd, env=_job_env()).decode().rstrip()
            self.slurm_ids.append(int(out.split()[-1]))
            print(out)

    def wait_for_jobs(self, job_prefix=None):
        _poll_until_gone('squeue -u $USER | grep $USER', '', self.slurm_ids, False)


class LSFTask(BaseClusterTask):
    """Jobs submitted with bsub, polled with bjobs."""

    def submit_jobs(self, n_jobs, job_prefix=None):
        tc = self.get_task_config()
        paths = _Paths(self.tmp_folder, self.task_name, job_prefix)
        assert os.path.exists(paths.script()), paths.script()
        self.bsub_ids = []
        for j in range(n_jobs):
            cmd = "bsub -n %i -J %s_%i -We %i -o %s -e %s '%s %s'" % (
                tc.get("threads_per_job", 1), self.task_name, j, tc.get("time_limit", 60), paths.log(j), paths.err(j),
                paths.script(), paths.config(j))
            out = subprocess.check_output([cmd], shell=True, env=_job_env()).decode().rstrip()
            self.bsub_ids.append(int(out.split()[1].strip('<>')))
            print(out)

    def wait_for_jobs(self, job_prefix=None):
        _poll_until_gone('bjobs | grep $USER', 'No unfinished job found', self.bsub_ids, True)

    @staticmethod
    def parse_jobs(log_prefix, max_jobs):
        return [j for j in range(max_jobs) if parse_job_lsf(log_prefix + '%i.log' % j, j)]


class WorkflowBase(luigi.Task):
    """Chains tasks; its target is the last task's target."""
    tmp_folder = luigi.Parameter()
    max_jobs = luigi.IntParameter()
    config_dir = luigi.Parameter()
    target = luigi.Parameter()
    dependency = luigi.TaskParameter(default=DummyTask())

    _target_dict = {'lsf': 'LSF', 'slurm': 'Slurm', 'local': 'Local'}

    def _get_task_name(self, task_base_name):
        return task_base_name + self._target_dict[self.target.lower()]

    def output(self):
        return luigi.LocalTarget(self.input().path)

    @staticmethod
    def get_config():
        return {'global': BaseClusterTask.default_global_config()}
