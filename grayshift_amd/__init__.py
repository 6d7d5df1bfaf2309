"""grayshift_amd — MI355X-native path-tracing hot path of benjisu03/grayshift.

The product is ``libgrayshift.so``: a persistent-wavefront HIP megakernel for gfx950
behind the C-ABI of include/grayshift_gpu.h, plus a C++ host mirror of the
reference's Camera / Hittable / Material surface (include/grayshift_host.h).

The public names below load that library on first use and raise if it is missing
(build it with ``python -m grayshift_amd.build``); there is no CPU fallback.
``grayshift_amd.build`` itself imports without the library.
"""
import importlib

_EXPORTS = {
    "HostScene": "renderer", "Renderer": "renderer", "camera": "renderer", "render": "renderer",
    "set_tuning": "renderer", "write_ppm": "renderer", "render_ppm": "renderer", "ppm_encode_async": "renderer",
    "render_multi": "renderer", "MultiRenderer": "renderer",
    "SceneBuilder": "scene", "camera_spec": "scene", "fixed_spp": "scene", "sample_settings": "scene",
}
_SUBMODULES = {"scenes", "partition", "assets", "_native", "scene", "codeobj"}

__all__ = sorted(_EXPORTS) + ["scenes"]


def __getattr__(name):
    if name in _EXPORTS:
        mod = importlib.import_module("." + _EXPORTS[name], __name__)
        return getattr(mod, name)
    if name in _SUBMODULES:
        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)
