"""JSON scene loading with the reference's schema, defaults, messages and error behaviour
(provided/scene_parser.py:50-294), returning an ``rtx.scene.Scene`` that renders on the GPU.

The reference parses with one function per JSON level; here the schema is data — the
optional camera sections, material keys and light kinds are tables — and every geometry
entry, at any depth, goes through one recursive builder (``_SceneBuilder.add``). What is
kept from the reference, because renders depend on it (tests/test_host.py,
tests/test_reference_binding.py compare against the reference's own parser):

* a section (AA, DOF, motion) with any key missing falls back as a whole (:67-96);
* a KeyError anywhere in the light list drops every light (:104-125); directional
  lights get power 1.0 whatever the JSON says (:116-118);
* material lists are ``associate_material``'s: for each listed ID, every scene material
  with that ID, in scene order (:288-294);
* a child's speed is its top-level hierarchy's speed plus its own, and nested nodes
  hand the TOP-LEVEL speed (not their own) to their children (:268-271, :283); a child
  of type "node" never resolves ``ref``;
* a top-level ``ref`` node deep-copies the first earlier root of that name and takes
  its own name, materials and transform (:190-205);
* every top-level hierarchy appends its materials to its leaves afterwards (:153-155);
* unknown light / object types are skipped with the reference's message.

``load_scene`` also accepts an already-parsed dict (the bench and tests use this); asset
paths that do not exist relative to the CWD are looked up next to the scene file.
"""
import copy
import json
import os

from . import f32 as F
from . import geometry as geom
from . import helperclasses as hc
from .scene import Scene
from .track import TList

# Optional camera sections: (JSON key, fields, fallbacks, message). A missing section or
# field takes every fallback of the section (scene_parser.py:67-96).
_SECTIONS = (
    ("AA", ("jitter", "samples"), (False, 1), "No Anti-Aliasing options found, setting to default"),
    ("DOF", ("focal_length", "aperture", "samples"), (1, 0, 1), "No Depth of Field options found, setting to default"),
    ("motion", ("time", "samples", "final"), (0, 1, 0), "No motion blur options found, setting to default"),
)

# Optional material keys in Material's argument order after (name, ID) (scene_parser.py:133-138).
_MATERIAL_KEYS = (("specular", [0, 0, 0]), ("diffuse", [0, 0, 0]), ("hardness", 32), ("type", "diffuse"),
                  ("tint", 0.0))

# Light kinds: JSON key of the light's vector and how its power is read (scene_parser.py:112-118).
_LIGHT_KINDS = {"point": ("position", lambda spec: spec["power"]),
                "directional": ("direction", lambda spec: 1.0)}


def _vec(a):
    """A JSON 3- or 4-list as a list, anything else of another length as None (the
    reference's populateVec, scene_parser.py:21-27)."""
    if a is None:
        return None
    return list(a) if len(a) in (3, 4) else None


class _Log:
    def __init__(self, verbose):
        self.verbose = verbose

    def __call__(self, *a):
        if self.verbose:
            print(*a)


class _SceneBuilder:
    def __init__(self, data, base_dir, log):
        self.data, self.base_dir, self.log = data, base_dir, log
        self.materials = []
        self.roots = {}  # top-level hierarchies that `ref` nodes may copy, first definition wins

    # ------------------------------------------------------------ camera, lights, materials
    def optional(self, key, default, message):
        try:
            return self.data[key]
        except KeyError:
            self.log(message)
            return default

    def section(self, key, fields, fallbacks, message):
        try:
            return tuple(self.data[key][f] for f in fields)
        except KeyError:
            self.log(message)
            return fallbacks

    def camera(self):
        cam = self.data["camera"]
        pos, lookat, up, fov = _vec(cam["position"]), _vec(cam["lookAt"]), _vec(cam["up"]), cam["fov"]
        width, height = self.optional("resolution", [1080, 720], "No resolution found, defaulting to 1080x720.")
        self.ambient = _vec(self.optional("ambient", [0, 0, 0], "No ambient light defined, defaulting to [0, 0, 0]"))
        (self.jitter, self.samples), lens, motion = (self.section(*s) for s in _SECTIONS)
        return hc.ViewportCamera().set_viewport(width, height).set_camera(pos, lookat, up, fov) \
            .set_lens(*lens).set_motion(*motion)

    def lights(self):
        out = []
        try:
            for spec in self.data["lights"]:
                kind, name, colour = spec["type"], spec["name"], _vec(spec["colour"])
                if kind not in _LIGHT_KINDS:
                    self.log("Unkown light type", kind, ", skipping initialization")
                    continue
                key, power = _LIGHT_KINDS[kind]
                out.append(hc.Light(kind, name, colour, _vec(spec[key]), power(spec)))
        except KeyError as e:
            self.log("Error loading lights: ", e)
            out = []
        return out

    def read_materials(self):
        for spec in self.data["materials"]:
            name, ident = spec["name"], spec["ID"]
            specular, diffuse, hardness, kind, tint = (spec.get(k, d) for k, d in _MATERIAL_KEYS)
            m = hc.Material(name, _vec(specular), _vec(diffuse), hardness, ident, kind, tint)
            m.refr_index = spec.get("refr_index", 1.0)
            self.materials.append(m)
        return self.materials

    def materials_of(self, spec):
        return TList(m for i in spec.get("materials", []) for m in self.materials if m.ID == i)

    # ------------------------------------------------------------ geometry
    def asset(self, path):
        return geom.resolve_path(path, self.base_dir)

    def shape(self, kind, name, pos, mats, speed, spec):
        """The non-hierarchy geometry classes (scene_parser.py:212-258); None if ``kind``
        is not one of them."""
        if kind == "sphere":
            return geom.Sphere(name, kind, mats, pos, spec["radius"], speed)
        if kind == "plane":
            g = geom.Plane(name, kind, mats, pos, _vec(spec["normal"]), speed)
            if "texture" in spec:
                g.texture = geom.open_texture(spec["texture"], self.base_dir)
                g.texture_scale = spec.get("texture_scale", 1.0)
            return g
        if kind == "box":
            if "size" in spec:
                g = geom.AABB(name, kind, mats, pos, _vec(spec["size"]), speed)
            else:  # declared by its corners
                g = geom.AABB(name, kind, mats, pos, [0, 0, 0], speed)
                g.minpos, g.maxpos = F.vec3(_vec(spec["min"])), F.vec3(_vec(spec["max"]))
            if "texture" in spec:
                g.texture = geom.open_texture(spec["texture"], self.base_dir)
            return g
        if kind == "mesh":
            path = self.asset(spec["filepath"])
            return geom.Mesh(name, kind, mats, pos, spec["scale"], path, spec.get("flat_shaded", False), speed)
        return None

    def add(self, spec, into, top_speed=None, nested=False):
        """Build one geometry entry into ``into``: a top-level object (nested=False) or a
        child of a hierarchy whose top-level speed is ``top_speed``."""
        name, kind = spec["name"], spec["type"]
        pos = _vec(spec.get("position", [0, 0, 0]))
        mats = self.materials_of(spec)
        if not nested:
            speed = _vec(spec.get("speed"))
        elif top_speed is None:
            speed = None
        else:
            speed = F.vec3(top_speed) + F.vec3(_vec(spec.get("speed", [0, 0, 0])))
        g = self.shape(kind, name, pos, mats, speed, spec)
        if g is not None:
            into.append(g)
            return
        if kind != "node":
            if nested:  # the reference re-reads the entry as a top-level one, then skips it
                _vec(spec.get("speed"))
            self.log("Unkown object type", kind, ", skipping initialization")
            return
        ref = "" if nested else spec.get("ref", "")
        rot, scale = _vec(spec.get("rotation", [0, 0, 0])), _vec(spec.get("scale", [1, 1, 1]))
        htype = spec.get("hierarchy_type", "union")
        if ref != "":
            if ref not in self.roots:
                self.log("Node reference", ref, "not found, skipping creation")
                return
            node = copy.deepcopy(self.roots[ref])
            node.name, node.materials = name, mats
            node.make_matrices(pos, rot, scale)
            into.append(node)
            return
        node = geom.Hierarchy(name, kind, mats, htype, pos, rot, scale, speed)
        # children see the TOP-LEVEL speed, however deep (scene_parser.py:283)
        child_speed = top_speed if nested else speed
        for child in spec["children"]:
            self.add(child, node.children, child_speed, nested=True)
        if not nested:
            self.roots.setdefault(name, node)
        into.append(node)

    def objects(self):
        out = []
        for spec in self.data["objects"]:
            self.add(spec, out)
        for g in out:  # hierarchy.py:21-28, for top-level hierarchies only
            if isinstance(g, geom.Hierarchy):
                g.set_fallback_material(g.materials)
        return out


def load_scene(infile, verbose=True):
    """scene_parser.load_scene: a scene JSON file (or its parsed dict) -> Scene."""
    log = _Log(verbose)
    base_dir = None
    if isinstance(infile, dict):
        data = infile
    else:
        log("Parsing file:", infile)
        with open(infile) as f:
            data = json.load(f)
        base_dir = os.path.dirname(os.path.abspath(infile))
    b = _SceneBuilder(data, data.get("__base_dir__", base_dir), log)
    vc = b.camera()
    lights = b.lights()
    materials = b.read_materials()
    objects = b.objects()
    log("Parsing complete")
    # the scene's own lists, tracked (rtx.track): edits between renders are re-uploaded
    sc = Scene(vc, b.jitter, b.samples, b.ambient, TList(lights), TList(materials), TList(objects))
    for g in objects:
        g.set_scene(sc)
    return sc
