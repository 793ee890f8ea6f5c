"""Import shim for the package directory ``task-vector-replication_amd/``
(its name is not a Python identifier).  ``import tvr_amd`` yields the package
itself; submodules are reachable as attributes and as ``tvr_amd.<name>``."""
import importlib.util
import pathlib
import sys

_NAME = "task_vector_replication_amd"
_DIR = pathlib.Path(__file__).resolve().parent / "task-vector-replication_amd"


def _load():
    if _NAME in sys.modules:
        return sys.modules[_NAME]
    spec = importlib.util.spec_from_file_location(_NAME, _DIR / "__init__.py",
                                                  submodule_search_locations=[str(_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[_NAME] = mod
    spec.loader.exec_module(mod)
    return mod


_pkg = _load()
for _sub in _pkg.SUBMODULES:
    sys.modules[f"{__name__}.{_sub}"] = getattr(_pkg, _sub)
sys.modules[__name__] = _pkg
