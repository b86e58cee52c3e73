"""Generate the committed input/expected-output fixtures from the reference's data files.

Runs ONLY in the build container, where the read-only reference snapshot is mounted at
/root/reference. It copies *data* (scene JSON dictionaries, the torus OBJ mesh and the
published renders) — no reference source code — into:

- ``assets/scenes.json``      all scene dictionaries, keyed by scene name. Mesh paths are
                              rewritten to the bundled mesh (``assets/torus_mesh.obj``).
- ``assets/torus_mesh.obj``   the reference's ``meshes/torus.obj`` (64 v, 128 f).
- ``tests/golden/published/<Name>.png``  the reference's published renders
                              (``renders/*.png``): the expected outputs the oracle is
                              pinned against.

Usage: ``python tests/golden/make_fixtures.py`` (idempotent).
"""
import json
import os
import shutil
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ASSETS = os.path.join(REPO, "assets")

# scene name -> reference JSON path. TorusMesh comes from test_scenes/ because
# scenes/TorusMesh.json points at a bunny.obj that the snapshot does not contain
# (test_scenes/TorusMesh.json:36,39).
SCENES = {
    "TwoSpheresPlane": "scenes/TwoSpheresPlane.json",
    "MirrorRefraction": "scenes/MirrorRefraction.json",
    "DepthOfField": "scenes/DepthOfField.json",
    "MotionBlur": "scenes/MotionBlur.json",
    "TorusMesh": "test_scenes/TorusMesh.json",
    "NovelScene1": "scenes/NovelScene1.json",
    "NovelScene2": "scenes/NovelScene2.json",
}

RENDERS = ["TwoSpheresPlane", "MirrorRefraction", "MotionBlur", "TorusMesh",
           "TorusMesh_flat", "DepthOfField"]


def main():
    if not os.path.isdir(REF):
        sys.exit("reference snapshot not mounted; fixtures are already committed")
    os.makedirs(ASSETS, exist_ok=True)
    out = {}
    for name, rel in SCENES.items():
        with open(os.path.join(REF, rel)) as f:
            sc = json.load(f)
        for obj in sc.get("objects", []):
            if obj.get("type") == "mesh" and obj.get("filepath", "").endswith("torus.obj"):
                obj["filepath"] = "torus_mesh.obj"
        out[name] = sc
    with open(os.path.join(ASSETS, "scenes.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    shutil.copyfile(os.path.join(REF, "meshes/torus.obj"), os.path.join(ASSETS, "torus_mesh.obj"))
    pub = os.path.join(HERE, "published")
    os.makedirs(pub, exist_ok=True)
    for r in RENDERS:
        shutil.copyfile(os.path.join(REF, "renders", r + ".png"), os.path.join(pub, r + ".png"))
    print("wrote", os.path.join(ASSETS, "scenes.json"), "and", len(RENDERS), "published renders")


if __name__ == "__main__":
    main()
