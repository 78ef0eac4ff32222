from .chunked import File, Dataset, Group  # noqa: F401
