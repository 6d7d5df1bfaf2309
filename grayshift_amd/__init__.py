"""grayshift_amd — MI355X-native path-tracing hot path of benjisu03/grayshift.

The product is ``libgrayshift.so``: a persistent-wavefront HIP megakernel for gfx950
behind the C-ABI of include/grayshift_gpu.h, plus a C++ host mirror of the
reference's Camera / Hittable / Material surface (include/grayshift_host.h).
Importing this package loads that library and raises if it is missing; there is no
CPU fallback.
"""
from . import _native  # noqa: F401  (loads libgrayshift.so or raises)
from .render import HostScene, Renderer, camera, render, set_tuning, write_ppm  # noqa: F401
from .scene import SceneBuilder, camera_spec, fixed_spp, sample_settings  # noqa: F401
from . import scenes  # noqa: F401

__all__ = ["HostScene", "Renderer", "camera", "render", "set_tuning", "write_ppm", "SceneBuilder",
           "camera_spec", "fixed_spp", "sample_settings", "scenes"]
