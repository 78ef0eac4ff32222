from .watershed_workflow import WatershedWorkflow  # noqa: F401
