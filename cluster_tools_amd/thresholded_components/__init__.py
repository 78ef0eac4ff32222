from .thresholded_components_workflow import ThresholdedComponentsWorkflow, ThresholdAndWatershedWorkflow  # noqa: F401
