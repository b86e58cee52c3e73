"""Host I/O: bundled scenes and PNG output (main.py:30-35, glue.py:17-27)."""
import copy
import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ASSETS = os.path.join(REPO, "assets")


def bundled_scene_dict(name, resolution=None, spp=None, **edits):
    """A scene dictionary from assets/scenes.json, with the JSON edits the bench configs
    use: ``resolution=(W, H)``, ``spp=(aa, dof)`` or other top-level keys."""
    with open(os.path.join(ASSETS, "scenes.json")) as f:
        data = copy.deepcopy(json.load(f)[name])
    if resolution is not None:
        data["resolution"] = [int(resolution[0]), int(resolution[1])]
    if spp is not None:
        aa, dof = spp
        data.setdefault("AA", {"jitter": False, "samples": 1})
        data["AA"]["samples"] = int(aa)
        if dof is not None:
            data.setdefault("DOF", {"focal_length": 1, "aperture": 0, "samples": 1})
            data["DOF"]["samples"] = int(dof)
    data.update(edits)
    data["__base_dir__"] = ASSETS
    return data


def load_bundled_scene(name, verbose=False, **kw):
    from .scene_parser import load_scene
    return load_scene(bundled_scene_dict(name, **kw), verbose=verbose)


def to_png_array(image):
    """main.py:31-33: rot90(k=1, axes=(0, 1)), then (image * 255).astype(uint8)."""
    return (np.rot90(image, k=1, axes=(0, 1)) * 255).astype(np.uint8)


def save_png(image, path):
    from PIL import Image
    Image.fromarray(to_png_array(image)).save(path)
