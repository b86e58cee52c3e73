"""rtx — MI355X-native drop-in for the render path of SpacewaIker/python-raytracer.

Host API (mirrors the reference's provided/*.py): ``load_scene`` (scene_parser.py),
``Scene.render`` (scene.py), the CLI in ``rtx.main`` (main.py) and ``rtx.glue`` (glue.py).
The per-pixel render loop and the intersectors run as HIP kernels in librtx.so.
"""
from .scene import Scene, split_rows, strip_columns  # noqa: F401
from .scene_parser import load_scene  # noqa: F401
from .io import load_bundled_scene, save_png, to_png_array  # noqa: F401
from ._native import get_option, option_names, set_option  # noqa: F401

__all__ = ["Scene", "load_scene", "load_bundled_scene", "save_png", "to_png_array", "split_rows", "strip_columns",
           "set_option", "get_option", "option_names"]
