"""Cluster task runtime of the watershed path: config files, job configs, job scripts,
submission, log-based success checks and block-level retry.

Same contract as cluster_tools/cluster_tasks.py:25-654, which callers and the job scripts rely on:
* configs: ``config_dir/global.config`` and ``config_dir/<task_name>.config``, used verbatim
  when present (no merge with the defaults, :172-224);
* job configs: ``tmp_folder/<task_name>_job_[<prefix>_]<id>.config`` = task config +
  ``block_list`` (= ``block_list[job::n_jobs]``, :298-332);
* job scripts: the task module copied to ``tmp_folder/<task_name>.py`` with the configured
  shebang (:352-372), run with the job config path;
* logs: stdout -> ``tmp_folder/logs/<job_name>_<id>.log``, stderr -> ``error_logs``; a job
  succeeded iff its last line is ``processed job <id>``; failed blocks are the scheduled blocks
  not logged as ``processed block <id>``; retry while ``n_retries < max_num_retries``, the
  task allows it and < 50 % of jobs failed, else rename the task log to ``*_failed.log`` and
  raise FailedJobsError (:112-170);
* luigi target: ``tmp_folder/<task_name>.log`` (:247-248).

GPU jobs: a LocalTask job process opens one libctws handle on GPU ``job_id % n_gpus`` (set as
CTWS_DEVICE in the job environment), so ``max_jobs`` jobs share the node's GPUs.
"""
import fileinput
import json
import os
import shutil
import stat
import subprocess
import sys
import time
from concurrent import futures
from datetime import datetime, timedelta
from multiprocessing import cpu_count
from subprocess import call, check_output, CalledProcessError, STDOUT

import numpy as np

from . import luigi_compat as luigi
from .utils.parse_utils import parse_blocks_task, parse_job, parse_job_lsf
from .utils.task_utils import DummyTask

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FailedJobsError(Exception):
    pass


def _job_env(job_id=None):
    """Environment of a job process: the package importable, one GPU per job."""
    env = dict(os.environ)
    pp = env.get('PYTHONPATH', '')
    if _PKG_ROOT not in pp.split(os.pathsep):
        env['PYTHONPATH'] = _PKG_ROOT + (os.pathsep + pp if pp else '')
    if job_id is not None and 'CTWS_DEVICE' not in os.environ:
        n_gpus = _count_gpus()
        if n_gpus > 0:
            env['CTWS_DEVICE'] = str(job_id % n_gpus)
    return env


def _count_gpus():
    vis = os.environ.get('HIP_VISIBLE_DEVICES', os.environ.get('CUDA_VISIBLE_DEVICES'))
    if vis is not None:
        return len([v for v in vis.split(',') if v.strip() != ''])
    try:
        return len([d for d in os.listdir('/dev/dri') if d.startswith('renderD')])
    except OSError:
        return 0


class BaseClusterTask(luigi.Task):
    """Base of a task that runs as jobs on the cluster.  Subclasses implement run_impl:
    global_config_values -> init -> get_task_config -> prepare_jobs -> submit_jobs ->
    wait_for_jobs -> check_jobs."""
    tmp_folder = luigi.Parameter()
    max_jobs = luigi.IntParameter()
    config_dir = luigi.Parameter()
    allow_retry = True
    n_retries = 0

    # ---- API -----------------------------------------------------------------------------
    def run(self):
        self.make_dirs()
        self._write_log("Start task %s" % self.task_name)
        try:
            self.run_impl()
        except FailedJobsError:
            raise
        except Exception as e:
            out_path = self.output().path
            fail_path = out_path[:-4] + '_failed.log'
            self._write_log("task failed in `run_impl` with %s" % str(e))
            self._write_log("move log from %s to %s" % (out_path, fail_path))
            shutil.move(out_path, fail_path)
            raise
        self._write_log("Done task %s" % self.task_name)

    def init(self, shebang):
        self._write_script_file(shebang)

    @staticmethod
    def parse_jobs(log_prefix, max_jobs):
        return [job_id for job_id in range(max_jobs) if parse_job(log_prefix + '%i.log' % job_id, job_id)]

    def _job_name(self, job_prefix=None):
        return self.task_name if job_prefix is None else '%s_%s' % (self.task_name, job_prefix)

    def check_jobs(self, n_jobs, job_prefix=None):
        log_prefix = os.path.join(self.tmp_folder, 'logs', '%s_' % self._job_name(job_prefix))
        success_list = self.parse_jobs(log_prefix, n_jobs)
        if len(success_list) == n_jobs:
            self._write_log("%s finished successfully" % self.task_name)
            return
        failed_jobs = set(range(n_jobs)) - set(success_list)
        self._write_log("%s failed for jobs:" % self.task_name)
        self._write_log("%s" % ', '.join(map(str, sorted(failed_jobs))))
        max_num_retries = self.get_global_config().get('max_num_retries', 0)
        retry = (self.n_retries < max_num_retries) and self.allow_retry
        retry = retry and len(failed_jobs) / n_jobs < 0.5
        if retry:
            failed_blocks = self.get_failed_blocks(n_jobs, success_list, job_prefix)
            self._write_log("resubmitting %i failed blocks in %i retry attempt" % (len(failed_blocks),
                                                                                   self.n_retries + 1))
            self.n_retries += 1
            self.block_list = failed_blocks
            self.run()
        else:
            out_path = self.output().path
            fail_path = out_path[:-4] + '_failed.log'
            self._write_log("move log from %s to %s" % (out_path, fail_path))
            shutil.move(out_path, fail_path)
            raise FailedJobsError("Task: %s failed for %i / %i jobs" % (self.task_name, len(failed_jobs), n_jobs))

    def get_failed_blocks(self, n_jobs, passed_jobs=(), job_prefix=None):
        """Scheduled blocks minus those logged as processed.  The reference iterates an empty
        list for the passed jobs' configs (cluster_tasks.py:159-163), so only the logs of
        failed jobs are parsed; blocks of passed jobs never re-run because they are not in
        ``self.block_list`` of the failed jobs... except that they are: we keep the reference
        behaviour and additionally add the passed jobs' block lists from their configs."""
        passed_blocks = []
        for job_id in passed_jobs:
            path = self._config_path(job_id, job_prefix)
            if os.path.exists(path):
                with open(path) as f:
                    passed_blocks.extend(json.load(f).get('block_list') or [])
        log_prefix = os.path.join(self.tmp_folder, 'logs', '%s_' % self._job_name(job_prefix))
        passed_blocks.extend(parse_blocks_task(log_prefix, n_jobs, passed_jobs))
        return sorted(set(self.block_list) - set(passed_blocks))

    def get_task_config(self):
        config_path = os.path.join(self.config_dir, self.task_name + '.config')
        if os.path.exists(config_path):
            self._write_log("reading task config from %s" % config_path)
            with open(config_path) as f:
                return json.load(f)
        self._write_log("reading default task config")
        return self.default_task_config()

    @staticmethod
    def default_task_config():
        return {'threads_per_job': 1, 'time_limit': 60, 'mem_limit': 1., 'qos': 'normal'}

    def get_global_config(self):
        config_path = os.path.join(self.config_dir, 'global.config')
        if os.path.exists(config_path):
            self._write_log("reading global config from %s" % config_path)
            with open(config_path) as f:
                return json.load(f)
        self._write_log("reading default global config")
        return self.default_global_config()

    @staticmethod
    def default_global_config():
        return {"block_shape": [50, 512, 512],
                "shebang": "#! /bin/python",
                "roi_begin": None,
                "roi_end": None,
                "groupname": "kreshuk",
                "partition": None,
                "max_num_retries": 0,
                "block_list_path": None}

    def global_config_values(self, with_block_list_path=False):
        config = self.get_global_config()
        conf = (config["shebang"], config["block_shape"], config.get("roi_begin", None),
                config.get("roi_end", None))
        if with_block_list_path:
            conf = conf + (config.get("block_list_path", None),)
        return conf

    def clean_up_for_retry(self, block_list, prefix=None):
        pass

    def output(self):
        return luigi.LocalTarget(os.path.join(self.tmp_folder, self.task_name + '.log'))

    # ---- must implement ------------------------------------------------------------------
    def prepare_jobs(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        raise NotImplementedError

    def submit_jobs(self, n_jobs, job_prefix=None):
        raise NotImplementedError

    def wait_for_jobs(self, job_prefix=None):
        raise NotImplementedError

    # ---- helpers -------------------------------------------------------------------------
    def _write_log(self, msg):
        with open(self.output().path, 'a') as f:
            f.write('%s: %s\n' % (str(datetime.now()), msg))

    def _config_path(self, job_id, job_prefix=None):
        if job_prefix is None:
            return os.path.join(self.tmp_folder, self.task_name + '_job_%s.config' % str(job_id))
        return os.path.join(self.tmp_folder, self.task_name + '_job_%s_%s.config' % (job_prefix, str(job_id)))

    def make_dirs(self):
        for d in (self.tmp_folder, os.path.join(self.tmp_folder, 'logs'),
                  os.path.join(self.tmp_folder, 'error_logs')):
            os.makedirs(d, exist_ok=True)
        self._write_log('created tmp-folder and log dirs @ %s' % self.tmp_folder)

    def _write_job_config(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        if block_list is None:
            assert n_jobs == 1
            with open(self._config_path(0, job_prefix), 'w') as f:
                json.dump(config, f)
        else:
            self.block_list = block_list
            if consecutive_blocks:
                per_job = np.zeros(n_jobs, dtype='uint32')
                for i in range(len(block_list)):
                    per_job[i % n_jobs] += 1
                bounds = np.concatenate([[0], np.cumsum(per_job)]).astype(int)
            for job_id in range(n_jobs):
                if consecutive_blocks:
                    block_jobs = list(range(bounds[job_id], bounds[job_id + 1]))
                else:
                    block_jobs = block_list[job_id::n_jobs]
                with open(self._config_path(job_id, job_prefix), 'w') as f:
                    json.dump({'block_list': block_jobs, **config}, f)
        self._write_log('written config for %i jobs' % n_jobs)

    def _write_script_file(self, shebang):
        assert os.path.exists(self.src_file), self.src_file
        trgt_file = os.path.join(self.tmp_folder, self.task_name + '.py')
        shutil.copy(self.src_file, trgt_file)
        for i, line in enumerate(fileinput.input(trgt_file, inplace=True)):
            print(shebang if i == 0 else line, end='' if i else '\n')
        st = os.stat(trgt_file)
        os.chmod(trgt_file, st.st_mode | stat.S_IEXEC)
        self._write_log('copied python script from %s to %s' % (self.src_file, trgt_file))


class SlurmTask(BaseClusterTask):
    """Jobs submitted with sbatch, polled with squeue (cluster_tasks.py:375-490)."""

    @staticmethod
    def _parse_time_limit(time_limit):
        tt = timedelta(minutes=time_limit) + datetime(1, 1, 1)
        return "%i-%i:%i:%i" % (tt.day - 1, tt.hour, tt.minute, tt.second)

    @staticmethod
    def _parse_mem_limit(mem_limit):
        return "%iG" % mem_limit if mem_limit > 1 else "%iM" % int(mem_limit * 1000)

    def _write_slurm_file(self, job_prefix=None):
        gc = self.get_global_config()
        tc = self.get_task_config()
        lines = ["#!/bin/bash", "#SBATCH -A %s" % gc.get('groupname', 'kreshuk'), "#SBATCH -N 1",
                 "#SBATCH -c %i" % tc.get("threads_per_job", 1),
                 "#SBATCH --mem %s" % self._parse_mem_limit(tc.get("mem_limit", 2)),
                 "#SBATCH -t %s" % self._parse_time_limit(tc.get("time_limit", 60)),
                 "#SBATCH --qos=%s" % tc.get("qos", "normal")]
        if gc.get('partition', None) is not None:
            lines.append("#SBATCH -p=%s" % gc['partition'])
        if tc.get('gpus_per_job', 0):
            lines.append("#SBATCH --gres=gpu:%i" % tc['gpus_per_job'])
        trgt_file = os.path.join(self.tmp_folder, self.task_name + '.py')
        lines.append("%s %s" % (trgt_file, self._config_path('$1', job_prefix)))
        with open(os.path.join(self.tmp_folder, 'slurm_%s.sh' % self._job_name(job_prefix)), 'w') as f:
            f.write("\n".join(lines))

    def prepare_jobs(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        self._write_job_config(n_jobs, block_list, config, job_prefix, consecutive_blocks)
        self._write_slurm_file(job_prefix)

    def submit_jobs(self, n_jobs, job_prefix=None):
        job_name = self._job_name(job_prefix)
        script_path = os.path.join(self.tmp_folder, 'slurm_%s.sh' % job_name)
        self.slurm_ids = []
        for job_id in range(n_jobs):
            out_file = os.path.join(self.tmp_folder, 'logs', '%s_%i.log' % (job_name, job_id))
            err_file = os.path.join(self.tmp_folder, 'error_logs', '%s_%i.err' % (job_name, job_id))
            command = ['sbatch', '-o', out_file, '-e', err_file, '-J', '%s_%i' % (job_name, job_id),
                       script_path, str(job_id)]
            outp = check_output(command, env=_job_env()).decode().rstrip()
            self.slurm_ids.append(int(outp.split()[-1]))
            print(outp)

    def wait_for_jobs(self, job_prefix=None):
        while True:
            time.sleep(10)
            try:
                outp = check_output(['squeue -u $USER | grep $USER'], shell=True).decode()
            except CalledProcessError as e:
                if e.output.decode().rstrip() == '':
                    break
                raise
            outp = [o for o in outp.split('\n') if o != '']
            if not outp or sum(int(o.split()[0]) in self.slurm_ids for o in outp) == 0:
                break


class LocalTask(BaseClusterTask):
    """Jobs run as local subprocesses from a process pool (cluster_tasks.py:493-533)."""
    max_local_jobs = cpu_count()

    def prepare_jobs(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        self._write_job_config(n_jobs, block_list, config, job_prefix, consecutive_blocks)

    def _submit(self, job_id, job_prefix):
        script_path = os.path.join(self.tmp_folder, self.task_name + '.py')
        config_file = self._config_path(job_id, job_prefix)
        assert os.path.exists(script_path) and os.path.exists(config_file)
        job_name = self._job_name(job_prefix)
        log_file = os.path.join(self.tmp_folder, 'logs', '%s_%i.log' % (job_name, job_id))
        err_file = os.path.join(self.tmp_folder, 'error_logs', '%s_%i.err' % (job_name, job_id))
        with open(log_file, 'w') as f_out, open(err_file, 'w') as f_err:
            call([script_path, config_file], stdout=f_out, stderr=f_err, env=_job_env(job_id))

    def submit_jobs(self, n_jobs, job_prefix=None):
        assert n_jobs <= self.max_local_jobs, \
            "Trying to submit %i local jobs but limit is %i. Did you forget to set the target to slurm or lsf?" % \
            (n_jobs, self.max_local_jobs)
        # threads, not processes: each job is its own OS process already
        with futures.ThreadPoolExecutor(n_jobs) as pp:
            tasks = [pp.submit(self._submit, job_id, job_prefix) for job_id in range(n_jobs)]
            [t.result() for t in tasks]

    def wait_for_jobs(self, job_prefix=None):
        pass


class LSFTask(BaseClusterTask):
    """Jobs submitted with bsub, polled with bjobs (cluster_tasks.py:536-620)."""

    def prepare_jobs(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        self._write_job_config(n_jobs, block_list, config, job_prefix, consecutive_blocks)

    def submit_jobs(self, n_jobs, job_prefix=None):
        tc = self.get_task_config()
        n_threads = tc.get("threads_per_job", 1)
        time_limit = tc.get("time_limit", 60)
        script_path = os.path.join(self.tmp_folder, self.task_name + '.py')
        assert os.path.exists(script_path), script_path
        self.bsub_ids = []
        job_name = self._job_name(job_prefix)
        for job_id in range(n_jobs):
            command = '%s %s' % (script_path, self._config_path(job_id, job_prefix))
            log_file = os.path.join(self.tmp_folder, 'logs', '%s_%i.log' % (job_name, job_id))
            err_file = os.path.join(self.tmp_folder, 'error_logs', '%s_%i.err' % (job_name, job_id))
            bsub = "bsub -n %i -J %s_%i -We %i -o %s -e %s '%s'" % (n_threads, self.task_name, job_id, time_limit,
                                                                   log_file, err_file, command)
            outp = check_output([bsub], shell=True, env=_job_env()).decode().rstrip()
            self.bsub_ids.append(int(outp.split()[1].lstrip('<').rstrip('>')))
            print(outp)

    def wait_for_jobs(self, job_prefix=None):
        while True:
            time.sleep(10)
            try:
                outp = check_output(['bjobs | grep $USER'], shell=True, stderr=STDOUT).decode()
            except CalledProcessError as e:
                if e.output.decode().rstrip() == 'No unfinished job found':
                    break
                raise
            outp = [o for o in outp.split('\n') if o != '']
            if not outp or sum(int(o.split()[0]) in self.bsub_ids for o in outp) == 0:
                break

    @staticmethod
    def parse_jobs(log_prefix, max_jobs):
        return [j for j in range(max_jobs) if parse_job_lsf(log_prefix + '%i.log' % j, j)]


class WorkflowBase(luigi.Task):
    """Chains tasks; the target is the last task's target (cluster_tasks.py:623-654)."""
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
