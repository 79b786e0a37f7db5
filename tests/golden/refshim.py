"""Import shim for running the read-only reference (``/root/reference``) on CPU in the build container.

Test infrastructure only: used by the ``gen_golden_*.py`` scripts that produce the committed ``.npz`` fixtures.
Nothing here ships, and nothing on the GPU box imports it (``/root/reference`` does not exist there).

What the shim does (oracle recipe):
  * a minimal ``gym`` package (``gym.Env`` + ``gym.spaces.Box/Discrete``) written to a temp dir, because gym is absent;
  * ``torch.Tensor.cuda`` / ``torch.nn.Module.cuda`` patched to identity (no GPU here);
  * modules loaded by file path under unique names (the reference reuses module names across directories);
  * cwd moved to a temp dir because three env modules create ``./experiments`` at import.
"""
import importlib.util
import os
import sys
import tempfile

REF = os.environ.get("FLOCK_REFERENCE", "/root/reference")

_GYM_INIT = "class Env(object):\n    pass\nfrom . import spaces\n"
_GYM_SPACES = (
    "import numpy as np\n"
    "class Box(object):\n"
    "    def __init__(self, low, high, shape=None, dtype=np.float32):\n"
    "        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype\n"
    "class Discrete(object):\n"
    "    def __init__(self, n):\n"
    "        self.n = n\n"
    "        self.shape = ()\n"
)

_installed = False
_tmp = None


def available() -> bool:
    return os.path.isdir(os.path.join(REF, "environments"))


def install():
    """Install the gym stub + cuda no-op patches. Idempotent."""
    global _installed, _tmp
    if _installed:
        return _tmp
    import torch

    _tmp = tempfile.mkdtemp(prefix="flock_refshim_")
    os.makedirs(os.path.join(_tmp, "gym"))
    with open(os.path.join(_tmp, "gym", "__init__.py"), "w") as f:
        f.write(_GYM_INIT)
    with open(os.path.join(_tmp, "gym", "spaces.py"), "w") as f:
        f.write(_GYM_SPACES)
    sys.path.insert(0, _tmp)
    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.nn.Module.cuda = lambda self, *a, **k: self
    os.chdir(_tmp)
    _installed = True
    return _tmp


def load(relpath: str, name: str):
    """Load ``/root/reference/<relpath>`` as module ``name`` (by file path, no sys.path collisions)."""
    install()
    path = os.path.join(REF, relpath)
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod
