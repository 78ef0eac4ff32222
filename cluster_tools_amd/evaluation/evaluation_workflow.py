"""EvaluationWorkflow: drop-in for cluster_tools/evaluation/evaluation_workflow.py:53-77
(seg_path/key, gt_path/key, output_path, ignore_label).  The reference's two stages
(NodeLabelWorkflow overlaps, then Measures) are one GPU job here (measures.GpuMeasures*);
the output JSON has the same keys.  ObjectViWorkflow (per-object VI) is not part of this build."""
from cluster_tools_amd import luigi_compat as luigi
from cluster_tools_amd.cluster_tasks import WorkflowBase
from cluster_tools_amd.evaluation import measures as measure_tasks


class EvaluationWorkflow(WorkflowBase):
    seg_path = luigi.Parameter()
    seg_key = luigi.Parameter()
    gt_path = luigi.Parameter()
    gt_key = luigi.Parameter()
    output_path = luigi.Parameter()
    ignore_label = luigi.BoolParameter(default=True)

    def requires(self):
        task = getattr(measure_tasks, self._get_task_name('GpuMeasures'))
        return task(tmp_folder=self.tmp_folder, config_dir=self.config_dir, max_jobs=self.max_jobs,
                    dependency=self.dependency, seg_path=self.seg_path, seg_key=self.seg_key,
                    gt_path=self.gt_path, gt_key=self.gt_key, output_path=self.output_path,
                    ignore_label=self.ignore_label)

    @staticmethod
    def get_config():
        configs = WorkflowBase.get_config()
        configs.update({'gpu_measures': measure_tasks.GpuMeasuresLocal.default_task_config()})
        return configs
