from .evaluation_workflow import EvaluationWorkflow  # noqa: F401
