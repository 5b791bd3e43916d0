"""Loader for the in-tree gfx950 extension ``unet_distributed_amd/_C*.so``.

``torch`` is imported first on purpose: the extension links ``libamdhip64.so.7``
by soname and must bind to the HIP runtime PyTorch already loaded (PyTorch
ships its own copy), never to a second one.

On a GPU machine the native path is mandatory: ``require()`` raises if the
extension is missing or fails to load, so nothing silently falls back to ATen.
"""

import os

import torch  # noqa: F401  (must precede the extension import)

_lib = None
_err = None


def _load():
    global _lib, _err
    if _lib is not None or _err is not None:
        return
    try:
        from .. import _C  # type: ignore
        _lib = _C
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e


def available() -> bool:
    _load()
    return _lib is not None


def lib():
    _load()
    if _lib is None:
        raise RuntimeError(
            "native extension unet_distributed_amd._C is not built or failed to load (%r); "
            "run `python -m unet_distributed_amd.native.build`" % (_err,))
    return _lib


def require():
    """Return the extension; raise loudly when it is missing (GPU path)."""
    return lib()


def build_if_needed(verbose=False):
    from .build import build
    return build(verbose=verbose)


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def disabled_by_env() -> bool:
    return os.environ.get("UNET_DISABLE_NATIVE", "0") == "1"
