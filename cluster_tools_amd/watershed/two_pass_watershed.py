#! /usr/bin/env python
"""Two-pass (checkerboard) watershed: drop-in for cluster_tools/watershed/two_pass_watershed.py.

Pass 0 runs `_ws_block` on the blocks of one checkerboard colour, pass 1 runs `_ws_pass2` on
the others, seeded by the pass-0 labels in their halo (two_pass_watershed.py:60-93, 210-255).
Both passes are libctws calls (cfg.pass_id); the checkerboard lists come from
utils.volume_utils.make_checkerboard_block_lists (volume_utils.py:142-205).
"""
import json
import os
import sys

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask
from cluster_tools_amd.watershed.watershed import run_blocks


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

    def _ws_pass(self, block_list, config, prefix):
        n_jobs = min(len(block_list), self.max_jobs)
        self.prepare_jobs(n_jobs, block_list, config, prefix)
        self.submit_jobs(n_jobs, prefix)
        self.wait_for_jobs(prefix)
        self.check_jobs(n_jobs, prefix)

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end, block_list_path = self.global_config_values(True)
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        if len(shape) == 4:
            shape = shape[1:]
        ws_config = self.get_task_config()
        chunks = tuple(bs // 2 for bs in block_shape)
        with vu.file_reader(self.output_path) as f:
            f.require_dataset(self.output_key, shape=shape, chunks=chunks, compression='gzip', dtype='uint64')
        ws_config.update({'input_path': self.input_path, 'input_key': self.input_key,
                          'output_path': self.output_path, 'output_key': self.output_key,
                          'block_shape': block_shape})
        if self.mask_path != '':
            assert self.mask_key != ''
            ws_config.update({'mask_path': self.mask_path, 'mask_key': self.mask_key})
        blocking = Blocking([0, 0, 0], list(shape), list(block_shape))
        block_lists = vu.make_checkerboard_block_lists(blocking, roi_begin, roi_end)
        for pass_id, block_list in enumerate(block_lists):
            ws_config['pass'] = pass_id
            self._ws_pass(block_list, ws_config, 'pass_%i' % pass_id)


class TwoPassWatershedLocal(TwoPassWatershedBase, LocalTask):
    pass


class TwoPassWatershedSlurm(TwoPassWatershedBase, SlurmTask):
    pass


class TwoPassWatershedLSF(TwoPassWatershedBase, LSFTask):
    pass


def two_pass_watershed(job_id, config_path):
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    shape = list(vu.get_shape(config['input_path'], config['input_key']))
    if len(shape) == 4:
        shape = shape[1:]
    block_shape = list(config['block_shape'])
    blocking = Blocking([0, 0, 0], shape, block_shape)
    pass_id = config['pass']
    with vu.file_reader(config['input_path'], 'r') as f_in, vu.file_reader(config['output_path']) as f_out:
        ds_in = f_in[config['input_key']]
        assert ds_in.ndim in (3, 4)
        ds_out = f_out[config['output_key']]
        assert ds_out.ndim == 3
        mask = vu.load_mask(config['mask_path'], config['mask_key'], shape) if 'mask_path' in config else None
        run_blocks(blocking, config['block_list'], ds_in, ds_out, mask, config, pass_id=pass_id)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    two_pass_watershed(job_id, path)
