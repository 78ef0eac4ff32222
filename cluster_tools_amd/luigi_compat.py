"""luigi, or a minimal luigi-compatible shim when luigi is not installed.

The reference task surface is luigi (cluster_tools/cluster_tasks.py, watershed/*.py).  luigi is
not installed in this image and cannot be fetched, so this module re-exports real luigi when it
is importable and otherwise provides the subset the task surface uses:
Task / WrapperTask, Parameter, IntParameter, FloatParameter, BoolParameter, ListParameter,
DictParameter, TaskParameter, LocalTarget and build(tasks, local_scheduler=True) with luigi's
completion semantics (a task is complete iff all its outputs exist) and dependency order.
"""
try:  # pragma: no cover - exercised only where luigi is installed
    import luigi as _luigi
    Task = _luigi.Task
    WrapperTask = _luigi.WrapperTask
    Parameter = _luigi.Parameter
    IntParameter = _luigi.IntParameter
    FloatParameter = _luigi.FloatParameter
    BoolParameter = _luigi.BoolParameter
    ListParameter = _luigi.ListParameter
    DictParameter = _luigi.DictParameter
    TaskParameter = _luigi.TaskParameter
    LocalTarget = _luigi.LocalTarget
    build = _luigi.build
    HAVE_LUIGI = True
except ImportError:
    import os
    import traceback

    HAVE_LUIGI = False
    _NODEFAULT = object()

    class Parameter:
        _counter = 0

        def __init__(self, default=_NODEFAULT, **kwargs):
            self.default = default
            Parameter._counter += 1
            self._order = Parameter._counter

        def normalize(self, x):
            return x

    class IntParameter(Parameter):
        def normalize(self, x):
            return int(x)

    class FloatParameter(Parameter):
        def normalize(self, x):
            return float(x)

    class BoolParameter(Parameter):
        def __init__(self, default=False, **kwargs):
            super().__init__(default=default, **kwargs)

        def normalize(self, x):
            return bool(x)

    class ListParameter(Parameter):
        def normalize(self, x):
            return tuple(x) if isinstance(x, list) else x

    class DictParameter(Parameter):
        pass

    class TaskParameter(Parameter):
        pass

    class LocalTarget:
        def __init__(self, path):
            self.path = path

        def exists(self):
            return os.path.exists(self.path)

    class Task:
        """Parameters are class attributes; instances hold their values as attributes."""

        def __init__(self, **kwargs):
            params = self.get_params()
            for name, p in params:
                if name in kwargs:
                    val = p.normalize(kwargs.pop(name))
                elif p.default is not _NODEFAULT:
                    val = p.default
                else:
                    raise TypeError("%s: missing parameter %s" % (type(self).__name__, name))
                object.__setattr__(self, name, val)
            if kwargs:
                raise TypeError("%s: unknown parameters %s" % (type(self).__name__, sorted(kwargs)))

        @classmethod
        def get_params(cls):
            seen = {}
            for klass in reversed(cls.__mro__):
                for name, val in vars(klass).items():
                    if isinstance(val, Parameter):
                        seen[name] = val
            return sorted(seen.items(), key=lambda kv: kv[1]._order)

        def requires(self):
            return []

        def input(self):
            req = self.requires()
            if isinstance(req, Task):
                return req.output()
            if isinstance(req, (list, tuple)):
                return [r.output() for r in req]
            if isinstance(req, dict):
                return {k: r.output() for k, r in req.items()}
            return None

        def output(self):
            return []

        def complete(self):
            outs = self.output()
            if outs is None:
                return False
            if not isinstance(outs, (list, tuple)):
                outs = [outs]
            if len(outs) == 0:
                # tasks without outputs (WrapperTask) are complete when requirements are
                return all(r.complete() for r in _as_list(self.requires()))
            return all(o.exists() for o in outs)

        def run(self):
            pass

        def __repr__(self):
            return '%s(%s)' % (type(self).__name__, ', '.join('%s=%r' % (n, getattr(self, n))
                                                             for n, _ in self.get_params()))

    class WrapperTask(Task):
        def complete(self):
            return all(r.complete() for r in _as_list(self.requires()))

    def _as_list(req):
        if req is None:
            return []
        if isinstance(req, Task):
            return [req]
        if isinstance(req, dict):
            return list(req.values())
        return list(req)

    def _run(task, done):
        if id(task) in done or task.complete():
            done.add(id(task))
            return True
        for dep in _as_list(task.requires()):
            if not _run(dep, done):
                return False
        try:
            task.run()
        except Exception:
            traceback.print_exc()
            return False
        done.add(id(task))
        return True

    def build(tasks, local_scheduler=True, **kwargs):
        """Run the tasks and their requirements depth-first; True iff all succeeded."""
        done = set()
        ok = True
        for t in tasks:
            ok = _run(t, done) and ok
        return ok
