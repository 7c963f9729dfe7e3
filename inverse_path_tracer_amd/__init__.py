"""MI355X-native inverse path tracer (drop-in for bblinn2017/inverse_path_tracer's
ipt_cuda.py / libpt.so / libipt.so hot path).

    from inverse_path_tracer_amd import Scene
    scene = Scene.from_file("assets/scenes/0.txt")
    img = scene.render(512, 512, 64, max_bounces=4, seed=0)

Submodules: ``ipt_cuda`` (the reference's FFI module, drop-in), ``scene``
(scene files + native scene handle), ``torch_ops`` (autograd op over the HIP
kernels), ``distributed`` (row-band / frame sharding over torch.distributed).
"""
from ._native import NativeError, device_count  # noqa: F401
from .scene import ObjectSpec, Scene, compress, parse_scene_text, png_read, png_write, unpack_graph  # noqa: F401

__version__ = "0.1.0"
