"""Import shim: exposes the on-disk package ``climate-super-resolution_amd/`` as ``climsr_amd``.

The hyphenated directory name is not a valid Python identifier, so this shim points the
package ``__path__`` at it; every submodule (``climsr_amd.models.esrgan`` ...) is then
resolved from ``climate-super-resolution_amd/``.  Hydra ``_target_`` strings use these
dotted paths.
"""
import os as _os

_REAL = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "climate-super-resolution_amd")
__path__ = [_REAL]
_init = _os.path.join(_REAL, "__init__.py")
with open(_init) as _f:
    exec(compile(_f.read(), _init, "exec"))
