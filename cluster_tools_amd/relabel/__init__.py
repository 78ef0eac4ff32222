from .relabel_workflow import RelabelWorkflow  # noqa: F401
