"""RelabelWorkflow: FindUniques -> FindLabeling -> Write (in place by default)
(cluster_tools/relabel/relabel_workflow.py:10-73)."""
from cluster_tools_amd import luigi_compat as luigi
from cluster_tools_amd.cluster_tasks import WorkflowBase
from cluster_tools_amd.relabel import find_uniques as unique_tasks
from cluster_tools_amd.relabel import find_labeling as labeling_tasks
from cluster_tools_amd.write import write as write_tasks


class RelabelWorkflow(WorkflowBase):
    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    assignment_path = luigi.Parameter()
    assignment_key = luigi.Parameter()
    output_path = luigi.Parameter(default='')
    output_key = luigi.Parameter(default='')
    # not in the reference: per-block uniques written by the producing watershed task
    # (WatershedBase.uniques_path), so FindUniques skips reading those blocks
    uniques_path = luigi.Parameter(default='')

    def requires(self):
        unique_task = getattr(unique_tasks, self._get_task_name('FindUniques'))
        dep = unique_task(tmp_folder=self.tmp_folder, max_jobs=self.max_jobs, config_dir=self.config_dir,
                          input_path=self.input_path, input_key=self.input_key, dependency=self.dependency,
                          uniques_path=self.uniques_path)
        labeling_task = getattr(labeling_tasks, self._get_task_name('FindLabeling'))
        dep = labeling_task(tmp_folder=self.tmp_folder, max_jobs=self.max_jobs, config_dir=self.config_dir,
                            dependency=dep, input_path=self.input_path, input_key=self.input_key,
                            assignment_path=self.assignment_path, assignment_key=self.assignment_key)
        if self.output_path == '':
            out_path, out_key = self.input_path, self.input_key
        else:
            assert self.output_key != ''
            out_path, out_key = self.output_path, self.output_key
        write_task = getattr(write_tasks, self._get_task_name('Write'))
        return write_task(tmp_folder=self.tmp_folder, max_jobs=self.max_jobs, config_dir=self.config_dir,
                          input_path=self.input_path, input_key=self.input_key,
                          output_path=out_path, output_key=out_key,
                          assignment_path=self.assignment_path, assignment_key=self.assignment_key,
                          identifier='relabel', dependency=dep)

    @staticmethod
    def get_config():
        configs = WorkflowBase.get_config()
        configs.update({'find_uniques': unique_tasks.FindUniquesLocal.default_task_config(),
                        'find_labeling': labeling_tasks.FindLabelingLocal.default_task_config(),
                        'write': write_tasks.WriteLocal.default_task_config()})
        return configs
