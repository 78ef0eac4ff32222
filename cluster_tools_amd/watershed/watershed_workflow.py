"""WatershedWorkflow: drop-in for cluster_tools/watershed/watershed_workflow.py:10-69.

Watershed{Local,Slurm,LSF} (or TwoPassWatershed* with two_pass=True), then RelabelWorkflow
(FindUniques -> FindLabeling -> Write in place, assignment table at
output_path/'relabel_watershed').  One-pass runs with target 'local' fold the relabel into the
watershed jobs (relabel_in_job, default on): the jobs exchange their per-block id counts over a
process group and write the final ids, the table and maxId themselves (job_relabel.py); the
output, table and maxId are those of the three-task RelabelWorkflow.  With max_num_retries > 0 in
the global config the three tasks run instead, so that failed blocks are retried as in the
reference.  The optional
post-watershed agglomeration of the reference (agglomeration=True, nifty RAG + clustering) is out
of scope for this build and raises.
"""
import json
import os

from cluster_tools_amd import luigi_compat as luigi
from cluster_tools_amd.cluster_tasks import WorkflowBase
from cluster_tools_amd.watershed import watershed as watershed_tasks
from cluster_tools_amd.watershed import two_pass_watershed as two_pass_tasks
from cluster_tools_amd.relabel import RelabelWorkflow


class WatershedWorkflow(WorkflowBase):
    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    output_path = luigi.Parameter()
    output_key = luigi.Parameter()
    mask_path = luigi.Parameter(default='')
    mask_key = luigi.Parameter(default='')
    two_pass = luigi.BoolParameter(default=False)
    agglomeration = luigi.BoolParameter(default=False)
    # not in the reference: the relabel inside the local watershed jobs (see above)
    relabel_in_job = luigi.BoolParameter(default=True)

    def requires(self):
        if self.agglomeration:
            raise NotImplementedError("agglomeration=True (nifty RAG + agglomerative clustering) is not "
                                      "part of this build")
        if self.two_pass:
            ws_task = getattr(two_pass_tasks, self._get_task_name('TwoPassWatershed'))
        else:
            ws_task = getattr(watershed_tasks, self._get_task_name('Watershed'))
        # the in-job relabel numbers every block of the task at once, so a failed block cannot be
        # re-run on its own afterwards: with max_num_retries > 0 the three tasks run instead, so
        # that the watershed task keeps the reference's block-level retry (cluster_tasks.py:127-142)
        if self.relabel_in_job and not self.two_pass and self.target == 'local' and self._max_retries() == 0:
            return ws_task(tmp_folder=self.tmp_folder, max_jobs=self.max_jobs, config_dir=self.config_dir,
                           input_path=self.input_path, input_key=self.input_key,
                           output_path=self.output_path, output_key=self.output_key,
                           mask_path=self.mask_path, mask_key=self.mask_key,
                           assignment_path=self.output_path, assignment_key='relabel_watershed')
        # the watershed jobs keep the uniques of the blocks they write; FindUniques reads those
        # instead of the label volume
        uniques_path = os.path.join(self.tmp_folder, 'watershed_block_uniques')
        dep = ws_task(tmp_folder=self.tmp_folder, max_jobs=self.max_jobs, config_dir=self.config_dir,
                      input_path=self.input_path, input_key=self.input_key,
                      output_path=self.output_path, output_key=self.output_key,
                      mask_path=self.mask_path, mask_key=self.mask_key, uniques_path=uniques_path)
        return RelabelWorkflow(tmp_folder=self.tmp_folder, max_jobs=self.max_jobs, config_dir=self.config_dir,
                               target=self.target, input_path=self.output_path, input_key=self.output_key,
                               assignment_path=self.output_path, assignment_key='relabel_watershed',
                               dependency=dep, uniques_path=uniques_path)

    def _max_retries(self):
        path = os.path.join(self.config_dir, 'global.config')
        if not os.path.exists(path):
            return 0
        with open(path) as f:
            return int(json.load(f).get('max_num_retries', 0) or 0)

    @staticmethod
    def get_config():
        configs = WorkflowBase.get_config()
        configs.update({'watershed': watershed_tasks.WatershedLocal.default_task_config(),
                        'two_pass_watershed': two_pass_tasks.TwoPassWatershedLocal.default_task_config(),
                        **RelabelWorkflow.get_config()})
        return configs
