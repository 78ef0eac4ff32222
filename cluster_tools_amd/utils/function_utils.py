"""Job log protocol (cluster_tools/utils/function_utils.py:7-22).

Jobs write to stdout, which LocalTask/SlurmTask/LSFTask redirect into
tmp_folder/logs/<task>_<job>.log.  A job succeeded iff its last line is
"<datetime>: processed job <id>"; finished blocks are "<datetime>: processed block <id>".
"""
from datetime import datetime
from subprocess import check_output


def log(msg):
    print("%s: %s" % (str(datetime.now()), msg), flush=True)


def log_block_success(block_id):
    print("%s: processed block %i" % (str(datetime.now()), block_id), flush=True)


def log_job_success(job_id):
    print("%s: processed job %i" % (str(datetime.now()), job_id), flush=True)


def tail(path, n_lines):
    return check_output(['tail', '-%i' % n_lines, path]).decode().split('\n')[:-1]
