"""ThresholdedComponentsWorkflow and ThresholdAndWatershedWorkflow
(cluster_tools/thresholded_components/thresholded_components_workflow.py:17-144; same
parameters, task chain and config keys).

BlockComponents (GPU, k_threshcc.hip) -> MergeOffsets -> BlockFaces -> MergeAssignments
(boost_ufd representatives, libctws.so) -> Write in place with the offsets (GPU lookup) -- for
a local target folded into the BlockComponents jobs (merge_in_job.py, merge_in_job=True); the
threshold-and-watershed variant then grows the components as seeds with WatershedFromSeeds
(k_seeded.hip) into the same dataset.
"""
import os

from cluster_tools_amd import luigi_compat as luigi
from cluster_tools_amd.cluster_tasks import WorkflowBase
from cluster_tools_amd.utils import volume_utils as vu
from cluster_tools_amd.watershed import watershed_from_seeds as ws_tasks
from cluster_tools_amd.write import write as write_tasks
from cluster_tools_amd.thresholded_components import block_components as block_tasks
from cluster_tools_amd.thresholded_components import merge_offsets as offset_tasks
from cluster_tools_amd.thresholded_components import block_faces as face_tasks
from cluster_tools_amd.thresholded_components import merge_assignments as assignment_tasks


class ThresholdedComponentsWorkflow(WorkflowBase):
    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    output_path = luigi.Parameter()
    output_key = luigi.Parameter()
    assignment_key = luigi.Parameter()
    threshold = luigi.FloatParameter()
    threshold_mode = luigi.Parameter(default='greater')
    mask_path = luigi.Parameter(default='')
    mask_key = luigi.Parameter(default='')
    channel = luigi.Parameter(default=None)
    # local target: MergeOffsets -> BlockFaces -> MergeAssignments -> Write run inside the
    # BlockComponents jobs (merge_in_job.py), same outputs; False keeps the five-task chain
    merge_in_job = luigi.BoolParameter(default=True)

    def requires(self):
        block_task = getattr(block_tasks, self._get_task_name('BlockComponents'))
        offset_task = getattr(offset_tasks, self._get_task_name('MergeOffsets'))
        face_task = getattr(face_tasks, self._get_task_name('BlockFaces'))
        assignment_task = getattr(assignment_tasks, self._get_task_name('MergeAssignments'))
        write_task = getattr(write_tasks, self._get_task_name('Write'))
        shape = list(vu.get_shape(self.input_path, self.input_key))
        if self.channel is None:
            assert len(shape) == 3
        else:
            assert len(shape) == 4
            shape = shape[1:]
        offset_path = os.path.join(self.tmp_folder, 'cc_offsets.json')
        common = dict(tmp_folder=self.tmp_folder, config_dir=self.config_dir, max_jobs=self.max_jobs)
        if self.merge_in_job and self.target == 'local':
            return block_task(input_path=self.input_path, input_key=self.input_key,
                              output_path=self.output_path, output_key=self.output_key,
                              threshold=self.threshold, threshold_mode=self.threshold_mode,
                              mask_path=self.mask_path, mask_key=self.mask_key, channel=self.channel,
                              dependency=self.dependency, assignment_key=self.assignment_key,
                              offsets_path=offset_path, **common)
        dep = block_task(input_path=self.input_path, input_key=self.input_key,
                         output_path=self.output_path, output_key=self.output_key,
                         threshold=self.threshold, threshold_mode=self.threshold_mode,
                         mask_path=self.mask_path, mask_key=self.mask_key, channel=self.channel,
                         dependency=self.dependency, **common)
        dep = offset_task(shape=shape, save_path=offset_path, dependency=dep, **common)
        dep = face_task(input_path=self.output_path, input_key=self.output_key, offsets_path=offset_path,
                        dependency=dep, **common)
        dep = assignment_task(output_path=self.output_path, output_key=self.assignment_key, shape=shape,
                              offset_path=offset_path, dependency=dep, **common)
        # in place on the output dataset
        dep = write_task(input_path=self.output_path, input_key=self.output_key,
                         output_path=self.output_path, output_key=self.output_key,
                         assignment_path=self.output_path, assignment_key=self.assignment_key,
                         identifier='thresholded_components', offset_path=offset_path, dependency=dep, **common)
        return dep

    @staticmethod
    def get_config():
        configs = super(ThresholdedComponentsWorkflow, ThresholdedComponentsWorkflow).get_config()
        configs.update({'block_components': block_tasks.BlockComponentsLocal.default_task_config(),
                        'merge_offsets': offset_tasks.MergeOffsetsLocal.default_task_config(),
                        'block_faces': face_tasks.BlockFacesLocal.default_task_config(),
                        'merge_assignments': assignment_tasks.MergeAssignmentsLocal.default_task_config(),
                        'write': write_tasks.WriteLocal.default_task_config()})
        return configs


class ThresholdAndWatershedWorkflow(WorkflowBase):
    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    output_path = luigi.Parameter()
    output_key = luigi.Parameter()
    assignment_key = luigi.Parameter()
    threshold = luigi.FloatParameter()
    threshold_mode = luigi.Parameter(default='greater')
    mask_path = luigi.Parameter(default='')
    mask_key = luigi.Parameter(default='')
    channel = luigi.IntParameter(default=None)
    merge_in_job = luigi.BoolParameter(default=True)

    def requires(self):
        dep = ThresholdedComponentsWorkflow(tmp_folder=self.tmp_folder, max_jobs=self.max_jobs,
                                            merge_in_job=self.merge_in_job,
                                            config_dir=self.config_dir, target=self.target,
                                            input_path=self.input_path, input_key=self.input_key,
                                            output_path=self.output_path, output_key=self.output_key,
                                            assignment_key=self.assignment_key, threshold=self.threshold,
                                            threshold_mode=self.threshold_mode, mask_path=self.mask_path,
                                            mask_key=self.mask_key, channel=self.channel,
                                            dependency=self.dependency)
        ws_task = getattr(ws_tasks, self._get_task_name('WatershedFromSeeds'))
        return ws_task(tmp_folder=self.tmp_folder, max_jobs=self.max_jobs, config_dir=self.config_dir,
                       dependency=dep, input_path=self.input_path, input_key=self.input_key,
                       seeds_path=self.output_path, seeds_key=self.output_key,
                       output_path=self.output_path, output_key=self.output_key,
                       mask_path=self.mask_path, mask_key=self.mask_key)

    @staticmethod
    def get_config():
        configs = super(ThresholdAndWatershedWorkflow, ThresholdAndWatershedWorkflow).get_config()
        configs.update({'watershed_from_seeds': ws_tasks.WatershedFromSeedsLocal.default_task_config(),
                        **ThresholdedComponentsWorkflow.get_config()})
        return configs
