"""Restrict BLAS / OpenMP threads before numpy is imported in a job process
(cluster_tools/utils/numpy_utils.py:5-33).  GPU jobs keep the reference's behaviour."""
import os


def set_numpy_threads(n_threads):
    for var in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS', 'VECLIB_NUM_THREADS',
                'NUMEXPR_NUM_THREADS'):
        os.environ[var] = str(n_threads)
