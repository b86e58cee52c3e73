"""Generate tests/golden/refobjects.json: the object graphs the reference's own
scene_parser.load_scene (provided/scene_parser.py:50-163) builds for the bundled scenes,
serialized attribute by attribute (class names kept), so tests can rebuild
reference-shaped objects without the reference (it does not travel to the GPU box).

Runs only in the build container: imports /root/reference/provided as-is, with the
test-only PyGLM / libigl stand-ins of tests/refshim first on sys.path, from
/root/reference as the working directory (the JSON asset paths are CWD-relative).

usage: python tests/golden/make_refobjects.py [out.json]
"""
import contextlib
import io
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

# (fixture name, reference scene file, resolution): one entry per bundled scene
SCENES = [
    ("TwoSpheresPlane", "scenes/TwoSpheresPlane.json", (64, 48)),
    ("MirrorRefraction", "scenes/MirrorRefraction.json", (64, 36)),
    ("MotionBlur", "scenes/MotionBlur.json", (50, 40)),
    ("TorusMesh", "test_scenes/TorusMesh.json", (48, 48)),
    ("DepthOfField", "scenes/DepthOfField.json", (48, 36)),
    ("NovelScene1", "scenes/NovelScene1.json", (64, 32)),
    ("NovelScene2", "scenes/NovelScene2.json", (32, 16)),
]


def encoder(glm, image_names):
    memo = {}

    def enc(x):
        if x is None or isinstance(x, (bool, int, str)):
            return x
        if isinstance(x, float):
            return x
        if isinstance(x, np.floating):
            return {"__np__": x.dtype.name, "v": float(x)}
        if isinstance(x, np.integer):
            return int(x)
        if isinstance(x, glm._Vec):
            return {"__vec__": x.N, "v": [float(c) for c in x.a]}
        if isinstance(x, glm.mat4):
            return {"__mat4__": [float(c) for c in x.m.ravel()]}
        if isinstance(x, np.ndarray):
            return {"__nd__": x.dtype.name, "shape": list(x.shape), "v": x.ravel().tolist()}
        if isinstance(x, list):
            return [enc(v) for v in x]
        if isinstance(x, tuple):
            return {"__tuple__": [enc(v) for v in x]}
        if id(x) in memo:
            return {"__ref__": memo[id(x)]}
        k = len(memo)
        memo[id(x)] = k
        _keep.append(x)  # ids stay unique while encoding
        if type(x).__module__.startswith("PIL."):
            name = image_names.get(np.asarray(x).tobytes())
            assert name, "texture not among the scene's files"
            return {"__image__": name, "__id__": k}
        attrs = {a: enc(v) for a, v in vars(x).items() if a != "scene"}  # scene: set_scene's back-pointer
        return {"__obj__": type(x).__name__, "__module__": type(x).__module__, "__id__": k, "attrs": attrs}
    _keep = []
    return enc


def main(out):
    sys.path[:0] = [os.path.join(os.path.dirname(HERE), "refshim"), os.path.join(REF, "provided")]
    os.chdir(REF)
    import glm
    import scene_parser
    from PIL import Image
    image_names = {}
    for f in sorted(os.listdir(os.path.join(REF, "textures"))):
        image_names[np.asarray(Image.open(os.path.join(REF, "textures", f))).tobytes()] = f
    result = {}
    for name, path, res in SCENES:
        with open(path) as f:
            data = json.load(f)
        data["resolution"] = list(res)
        with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as t:
            json.dump(data, t)
        try:
            with contextlib.redirect_stdout(io.StringIO()):  # the parser prints defaults
                sc = scene_parser.load_scene(t.name)
        finally:
            os.unlink(t.name)
        result[name] = {"source": path, "resolution": list(res), "scene": encoder(glm, image_names)(sc)}
    with open(out, "w") as f:
        json.dump(result, f, separators=(",", ":"))
        f.write("\n")


if __name__ == "__main__":
    main(os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else os.path.join(HERE, "refobjects.json"))
