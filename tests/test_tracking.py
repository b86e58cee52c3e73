"""Edits between renders (rtx.track): the reference reads every object,
material and light on every render (provided/scene.py:86-88, :148, :161-164), so
rtx.Scene must re-upload an edited scene without an invalidate() call. CPU tests of the
host logic: which edits count the epoch up, which scenes are tracked, and when
Scene.native() re-creates the upload (rtx_scene_create replaced by a recorder; the GPU
test renders through it: tests/test_gpu_parity.py test_edits_between_renders_*)."""
import copy

import numpy as np
import pytest

import rtx
from rtx import records, track
from rtx import scene as S
from rtx.geometry import Hierarchy, Sphere
from rtx.helperclasses import Light, Material
from rtx.io import bundled_scene_dict


def _scene(name="TwoSpheresPlane"):
    return rtx.load_scene(bundled_scene_dict(name, resolution=(32, 24)), verbose=False)


def _bumps(fn):
    e = track.epoch()
    fn()
    return track.epoch() - e


def test_parsed_scenes_are_tracked():
    for name in ("TwoSpheresPlane", "MirrorRefraction", "TorusMesh", "DepthOfField", "NovelScene1"):
        sc = _scene(name)
        assert track.scene_tracked(sc.objects, sc.materials, sc.lights, sc.ambient), name


def test_edits_count_the_epoch_up_and_reads_do_not():
    sc = _scene()
    sph = next(g for g in sc.objects if isinstance(g, Sphere))
    mat, light = sc.materials[0], sc.lights[0]
    assert _bumps(lambda: sph.center.__setitem__(1, 0.5)) == 1
    assert _bumps(lambda: sph.center[:2].__setitem__(0, 0.25)) == 1  # through a view
    def iadd():
        mat.diffuse *= np.float32(0.5)
    assert _bumps(iadd) >= 1
    assert _bumps(lambda: setattr(light, "power", 0.25)) == 1
    assert _bumps(lambda: sph.materials.append(mat)) == 1
    assert _bumps(lambda: sc.objects.pop()) == 1
    assert _bumps(lambda: setattr(sc, "ambient", np.zeros(3, np.float32))) == 1
    assert isinstance(sc.ambient, track.TArray)
    # reads and arithmetic do not count
    assert _bumps(lambda: (sph.center + 1, float(sph.radius), mat.diffuse.max(), list(sc.objects),
                           records.scene_desc(sc.objects, sc.materials, sc.lights, sc.ambient))) == 0
    r = sph.center * 2
    assert type(r) is np.ndarray


def test_untracked_values_make_the_scene_compared_per_render():
    sc = _scene()
    assert track.scene_tracked(sc.objects, sc.materials, sc.lights, sc.ambient)
    sph = next(g for g in sc.objects if isinstance(g, Sphere))
    keep = sph.materials
    sph.materials = [sc.materials[0]]  # a plain list the caller may still change
    assert not track.scene_tracked(sc.objects, sc.materials, sc.lights, sc.ambient)
    sph.materials = keep
    assert track.scene_tracked(sc.objects, sc.materials, sc.lights, sc.ambient)
    plain = S.Scene(sc.vc, sc.jitter, sc.samples, sc.ambient, list(sc.lights), list(sc.materials), list(sc.objects))
    assert not track.scene_tracked(plain.objects, plain.materials, plain.lights, plain.ambient)
    m = Material("m", (0, 0, 0), (1, 1, 1), 1, 9)
    m.diffuse = object()  # another mutable type
    assert not track.is_tracked(m)


def test_hierarchy_children_and_deep_copies_are_tracked():
    sc = _scene("NovelScene1")
    node = next(g for g in sc.objects if isinstance(g, Hierarchy))
    assert isinstance(node.children, track.TList)
    assert _bumps(lambda: node.children[0].materials.append(sc.materials[0])) == 1
    assert _bumps(lambda: node.t.__setitem__(0, 1.0)) == 1
    cp = copy.deepcopy(node)
    assert track.is_tracked(cp) and isinstance(cp.children, track.TList)
    assert _bumps(lambda: cp.children[0].materials.pop()) == 1


class _Recorder:
    """Stands in for _NativeScene (no GPU here): records every rtx_scene_create."""
    made = []

    def __init__(self, desc):
        self.h = None
        self.device = 0
        self.desc = records.desc_bytes(desc)
        _Recorder.made.append(self)

    def close(self):
        pass


@pytest.fixture
def recorder(monkeypatch):
    _Recorder.made = []
    monkeypatch.setattr(S, "_NativeScene", _Recorder)
    monkeypatch.setattr(S.torch.cuda, "current_device", lambda: 0)
    return _Recorder.made


def test_native_reuploads_only_after_a_change(recorder):
    sc = _scene()
    for _ in range(3):
        sc.native()
    assert len(recorder) == 1
    g0 = sc._gen
    sph = next(g for g in sc.objects if isinstance(g, Sphere))
    sph.center[1] = sph.center[1] + np.float32(0.25)
    sc.native()
    assert len(recorder) == 2 and sc._gen != g0
    # an assignment of the same value counts the epoch up, but the records are equal
    sph.radius = float(sph.radius)
    sc.native()
    assert len(recorder) == 2
    sc.materials[0].diffuse[0] = np.float32(0.125)
    sc.native()
    sc.lights[0].power = 3.0
    sc.native()
    assert len(recorder) == 4
    # the uploads differ where the edits are
    assert recorder[1].desc[0] != recorder[0].desc[0]  # objects
    assert recorder[2].desc[1] != recorder[1].desc[1]  # materials
    assert recorder[3].desc[2] != recorder[2].desc[2]  # lights
    # an edit of an unrelated scene's objects moves the epoch, not the upload
    other = _scene()
    other.lights[0].power = 7.0
    sc.native()
    assert len(recorder) == 4


def test_untracked_scene_is_compared_every_render(recorder, monkeypatch):
    sc = _scene()
    plain = S.Scene(sc.vc, sc.jitter, sc.samples, sc.ambient, list(sc.lights), list(sc.materials), list(sc.objects))
    calls = []
    real = records.desc_digest
    monkeypatch.setattr(records, "desc_digest", lambda d: calls.append(1) or real(d))
    plain.native()
    plain.native()
    assert len(calls) == 2 and len(recorder) == 1
    # a light appended to the plain list (no hook) is still seen
    plain.lights.append(Light("point", "x", (1, 1, 1), (0, 5, 0), 1.0))
    plain.native()
    assert len(recorder) == 2
