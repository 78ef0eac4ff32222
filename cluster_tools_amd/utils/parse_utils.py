"""Parse job logs for success, processed blocks and runtimes
(cluster_tools/utils/parse_utils.py:14-154): the retry machinery of BaseClusterTask.check_jobs
relies on exactly these rules."""
import datetime
import os
from subprocess import CalledProcessError

import numpy as np

from .function_utils import tail


def _stamp(line):
    d, t = line.split()[:2]
    y, m, dd = map(int, d.split('-'))
    h, mi, s = map(float, t[:-1].split(':'))
    return datetime.datetime(y, m, dd, int(h), int(mi), int(s))


def parse_runtime(log_file):
    with open(log_file) as f:
        lines = [ll.strip('\n') for ll in f if ll.strip()]
    return (_stamp(lines[-1]) - _stamp(lines[0])).total_seconds()


def parse_runtime_task(log_prefix, max_jobs, return_summary=True):
    runtimes = []
    for job_id in range(max_jobs):
        path = log_prefix + '%i.log' % job_id
        if not os.path.exists(path):
            break
        runtimes.append(parse_runtime(path))
    if return_summary:
        return (np.mean(runtimes), np.std(runtimes), len(runtimes))
    return runtimes


def parse_job(log_file, job_id):
    """True iff the last log line (minus the datetime prefix) is 'processed job <id>'."""
    try:
        last_line = tail(log_file, 1)[0]
    except (IndexError, CalledProcessError):
        return False
    return " ".join(last_line.split()[2:]) == "processed job %i" % job_id


def parse_job_lsf(log_file, job_id):
    """LSF appends its own report to the log; stop at the '-----' separator."""
    if not os.path.exists(log_file):
        return False
    with open(log_file) as f:
        for ll in f:
            ll = ll.rstrip()
            if ll.startswith('---------------'):
                return False
            if " ".join(ll.split()[2:]) == "processed job %i" % job_id:
                return True
    return False


def parse_blocks(log_file):
    blocks = []
    with open(log_file) as f:
        for line in f:
            line = ' '.join(line.split()[2:])
            if line.startswith('processed block'):
                blocks.append(int(line.split()[-1]))
    return blocks


def parse_blocks_task(log_prefix, max_jobs, complete_job_list=()):
    blocks = []
    for job_id in range(max_jobs):
        if job_id in complete_job_list:
            continue
        log_file = log_prefix + '%i.log' % job_id
        if not os.path.exists(log_file):
            continue
        blocks.extend(parse_blocks(log_file))
    return blocks
