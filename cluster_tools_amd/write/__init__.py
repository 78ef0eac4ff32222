from .write import WriteLocal, WriteSlurm, WriteLSF  # noqa: F401
