"""Job-log parsing for the task runtime's success / retry checks.

Contract (the reference's utils/parse_utils.py:14-154, which BaseClusterTask.check_jobs and the
job scripts agree on): every log line is ``<date> <time>: <message>``; a job succeeded iff the
message of its last line is ``processed job <id>``; a block counts as done when some line's
message is ``processed block <id>``.  LSF appends its own report after a line of dashes, which
ends the job's part of the log.
"""
import datetime
import os

import numpy as np

_LSF_REPORT = '---------------'


def _lines(path):
    """Non-empty lines of a log (no trailing newline); [] if it does not exist."""
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return [ln.rstrip('\n') for ln in f if ln.strip()]


def _message(line):
    """The part of a log line after its two timestamp fields."""
    return ' '.join(line.split()[2:])


def _timestamp(line):
    day, clock = line.split()[:2]
    clock = clock.rstrip(':')
    y, mo, d = (int(v) for v in day.split('-'))
    hh, mm, ss = clock.split(':')
    return datetime.datetime(y, mo, d, int(hh), int(mm), int(float(ss)))


def parse_job(log_file, job_id):
    """True iff the job's last log line (as `tail -n 1` gives it) is ``processed job <job_id>``."""
    if not os.path.exists(log_file):
        return False
    with open(log_file) as f:
        lines = f.read().split('\n')
    if lines and lines[-1] == '':
        lines.pop()  # the final newline
    return bool(lines) and _message(lines[-1]) == 'processed job %i' % job_id


def parse_job_lsf(log_file, job_id):
    """LSF variant: the success message may be followed by the scheduler's report."""
    want = 'processed job %i' % job_id
    for line in _lines(log_file):
        if line.startswith(_LSF_REPORT):
            return False
        if _message(line) == want:
            return True
    return False


def parse_blocks(log_file):
    """Block ids the job logged as processed, in log order."""
    out = []
    for line in _lines(log_file):
        msg = _message(line)
        if msg.startswith('processed block'):
            out.append(int(msg.rsplit(None, 1)[-1]))
    return out


def parse_blocks_task(log_prefix, max_jobs, complete_job_list=()):
    """Processed blocks of jobs 0..max_jobs-1 (log ``<prefix><id>.log``), skipping the given jobs."""
    skip = set(complete_job_list)
    return [b for j in range(max_jobs) if j not in skip for b in parse_blocks(log_prefix + '%i.log' % j)]


def parse_runtime(log_file):
    """Seconds between the first and the last line of a job log."""
    lines = _lines(log_file)
    return (_timestamp(lines[-1]) - _timestamp(lines[0])).total_seconds()


def parse_runtime_task(log_prefix, max_jobs, return_summary=True):
    """Runtimes of the consecutive existing job logs; (mean, std, count) by default."""
    times = []
    for j in range(max_jobs):
        path = log_prefix + '%i.log' % j
        if not os.path.exists(path):
            break
        times.append(parse_runtime(path))
    return (np.mean(times), np.std(times), len(times)) if return_summary else times
