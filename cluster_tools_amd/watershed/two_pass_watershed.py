#! /usr/bin/env python
"""Two-pass (checkerboard) watershed: drop-in for cluster_tools/watershed/two_pass_watershed.py.

Pass 0 runs `_ws_block` on the blocks of one checkerboard colour, pass 1 runs `_ws_pass2` on
the others, seeded by the pass-0 labels in their halo (two_pass_watershed.py:60-93, 210-255).
Both passes are libctws calls (cfg.pass_id); the checkerboard lists come from
utils.volume_utils.make_checkerboard_block_lists (volume_utils.py:142-205).
"""
import os
import sys

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask
from cluster_tools_amd.watershed.watershed import run_job, ws_task_setup


class TwoPassWatershedBase(luigi.Task):
    task_name = 'two_pass_watershed'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    output_path = luigi.Parameter()
    output_key = luigi.Parameter()
    mask_path = luigi.Parameter(default='')
    mask_key = luigi.Parameter(default='')
    uniques_path = luigi.Parameter(default='')   # see WatershedBase.uniques_path

    @staticmethod
    def default_task_config():
        config = LocalTask.default_task_config()
        config.update({'threshold': .5,
                       'apply_dt_2d': True, 'pixel_pitch': None,
                       'apply_ws_2d': True, 'sigma_seeds': 2., 'size_filter': 25,
                       'sigma_weights': 2., 'halo': [0, 0, 0],
                       'channel_begin': 0, 'channel_end': None,
                       'agglomerate_channels': 'mean', 'alpha': 0.8,
                       'invert_inputs': False, 'non_maximum_suppression': True})
        return config

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        shape, ws_config = ws_task_setup(self, block_shape)
        # pass 0 then pass 1, each a full job round (two_pass_watershed.py:60-93)
        colours = vu.make_checkerboard_block_lists(Blocking([0, 0, 0], list(shape), list(block_shape)),
                                                   roi_begin, roi_end)
        for pass_id, blocks in enumerate(colours):
            self.run_jobs(min(len(blocks), self.max_jobs), blocks, dict(ws_config, **{'pass': pass_id}),
                          'pass_%i' % pass_id)


class TwoPassWatershedLocal(TwoPassWatershedBase, LocalTask):
    pass


class TwoPassWatershedSlurm(TwoPassWatershedBase, SlurmTask):
    pass


class TwoPassWatershedLSF(TwoPassWatershedBase, LSFTask):
    pass


def two_pass_watershed(job_id, config_path):
    run_job(job_id, config_path)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    two_pass_watershed(job_id, path)
