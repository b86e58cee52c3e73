"""JSON scene loader with the reference's schema, defaults and error behaviour
(mirror of provided/scene_parser.py:21-294).

``load_scene(infile)`` returns an ``rtx.scene.Scene`` whose ``render()`` runs on the GPU.
Defaults (scene_parser.py:62-142): resolution [1080, 720], ambient [0,0,0], AA
{jitter: False, samples: 1}, DOF {focal_length: 1, aperture: 0, samples: 1}, motion
{time: 0, samples: 1, final: 0}, material {type: diffuse, diffuse/specular: [0,0,0],
hardness: 32, tint: 0.0, refr_index: 1.0}; directional lights get power 1.0; a KeyError
inside the light list drops every light; unknown light/object types are skipped with a
message. Hierarchy nodes (scene_parser.py:177-205, :261-285) become ``geometry.Hierarchy``
trees, `ref` nodes deep-copy an earlier root, and every top-level hierarchy passes its
materials to its leaves (hierarchy.py:21-28). Textures are opened with PIL like the
reference. ``load_scene`` also accepts an already-parsed dict (used by the bench and tests).
"""
import copy
import json
import os

from . import geometry as geom
from . import helperclasses as hc
from .scene import Scene


class _Log:
    def __init__(self, verbose):
        self.verbose = verbose

    def __call__(self, *a):
        if self.verbose:
            print(*a)


def populateVec(array):
    """scene_parser.py:21-27 (vec4 inputs are kept as 4-lists; only hierarchies use them)."""
    if array is None:
        return None
    if len(array) == 3:
        return [array[0], array[1], array[2]]
    if len(array) == 4:
        return [array[0], array[1], array[2], array[3]]
    return None


def get_or(obj, keys, default, msg="", log=print):
    """scene_parser.py:30-47."""
    if not isinstance(keys, list) or len(keys) == 0:
        try:
            return obj[keys]
        except KeyError:
            if msg != "":
                log(msg)
            return default
    result = []
    try:
        for key in keys:
            result.append(obj[key])
        return result
    except KeyError:
        if msg != "":
            log(msg)
        return default


def load_scene(infile, verbose=True):
    """scene_parser.py:50-163."""
    log = _Log(verbose)
    base_dir = None
    if isinstance(infile, dict):
        data = infile
    else:
        log("Parsing file:", infile)
        with open(infile) as f:
            data = json.load(f)
        base_dir = os.path.dirname(os.path.abspath(infile))
    base_dir = data.get("__base_dir__", base_dir)

    cam_pos = populateVec(data["camera"]["position"])
    cam_lookat = populateVec(data["camera"]["lookAt"])
    cam_up = populateVec(data["camera"]["up"])
    cam_fov = data["camera"]["fov"]

    width, height = get_or(data, "resolution", [1080, 720], "No resolution found, defaulting to 1080x720.", log)
    ambient = populateVec(get_or(data, "ambient", [0, 0, 0],
                                 "No ambient light defined, defaulting to [0, 0, 0]", log))
    try:
        jitter = data["AA"]["jitter"]
        samples = data["AA"]["samples"]
    except KeyError:
        log("No Anti-Aliasing options found, setting to default")
        jitter, samples = False, 1
    try:
        focal_length = data["DOF"]["focal_length"]
        aperture = data["DOF"]["aperture"]
        dof_samples = data["DOF"]["samples"]
    except KeyError:
        log("No Depth of Field options found, setting to default")
        focal_length, aperture, dof_samples = 1, 0, 1
    try:
        motion_time = data["motion"]["time"]
        motion_samples = data["motion"]["samples"]
        motion_final = data["motion"]["final"]
    except KeyError:
        log("No motion blur options found, setting to default")
        motion_time, motion_samples, motion_final = 0, 1, 0

    vc = hc.ViewportCamera() \
        .set_viewport(width, height) \
        .set_camera(cam_pos, cam_lookat, cam_up, cam_fov) \
        .set_lens(focal_length, aperture, dof_samples) \
        .set_motion(motion_time, motion_samples, motion_final)

    lights = []
    try:
        for light in data["lights"]:
            l_type = light["type"]
            l_name = light["name"]
            l_colour = populateVec(light["colour"])
            if l_type == "point":
                l_vector = populateVec(light["position"])
                l_power = light["power"]
            elif l_type == "directional":
                l_vector = populateVec(light["direction"])
                l_power = 1.0
            else:
                log("Unkown light type", l_type, ", skipping initialization")
                continue
            lights.append(hc.Light(l_type, l_name, l_colour, l_vector, l_power))
    except KeyError as e:
        log("Error loading lights: ", e)
        lights = []

    materials = []
    for material in data["materials"]:
        mat_name = material["name"]
        mat_id = material["ID"]
        mat_type = get_or(material, "type", "diffuse")
        mat_diffuse = populateVec(get_or(material, "diffuse", [0, 0, 0]))
        mat_specular = populateVec(get_or(material, "specular", [0, 0, 0]))
        mat_hardness = get_or(material, "hardness", 32)
        mat_tint = get_or(material, "tint", 0.0)
        mat_refr_index = get_or(material, "refr_index", 1.0)
        m = hc.Material(mat_name, mat_specular, mat_diffuse, mat_hardness, mat_id, mat_type, mat_tint)
        m.refr_index = mat_refr_index
        materials.append(m)

    objects = []
    rootNames = []   # hierarchies other nodes may reference (scene_parser.py:147-149)
    roots = []
    for geometry in data["objects"]:
        parse_geometry(geometry, objects, rootNames, roots, materials, base_dir, log)

    for obj in objects:
        if isinstance(obj, geom.Hierarchy):
            obj.set_fallback_material(obj.materials)

    log("Parsing complete")
    sc = Scene(vc, jitter, samples, ambient, lights, materials, objects)
    for obj in objects:
        obj.set_scene(sc)
    return sc


def parse_geometry(geometry, objects, rootNames, roots, materials, base_dir=None, log=print):
    """scene_parser.py:166-209: basic shapes, hierarchy roots, and nodes that deep-copy an
    earlier root (`ref`) with their own materials and transform."""
    g_name = geometry["name"]
    g_type = geometry["type"]
    g_pos = populateVec(get_or(geometry, "position", [0, 0, 0]))
    g_mats = associate_material(materials, get_or(geometry, "materials", []))
    g_speed = populateVec(get_or(geometry, "speed", None))
    if add_basic_shape(g_name, g_type, g_pos, g_speed, g_mats, geometry, objects, base_dir):
        return
    if g_type == "node":
        g_ref = get_or(geometry, "ref", "")
        g_r = populateVec(get_or(geometry, "rotation", [0, 0, 0]))
        g_s = populateVec(get_or(geometry, "scale", [1, 1, 1]))
        g_hierarchy_type = get_or(geometry, "hierarchy_type", "union")
        if g_ref == "":
            rootNames.append(g_name)
            node = geom.Hierarchy(g_name, g_type, g_mats, g_hierarchy_type, g_pos, g_r, g_s, g_speed)
            traverse_children(node, geometry["children"], materials, rootNames, roots, g_speed, base_dir, log)
            roots.append(node)
            objects.append(node)
        else:
            rid = rootNames.index(g_ref) if g_ref in rootNames else -1
            if rid != -1:
                node = copy.deepcopy(roots[rid])
                node.name = g_name
                node.materials = g_mats
                node.make_matrices(g_pos, g_r, g_s)
                objects.append(node)
            else:
                log("Node reference", g_ref, "not found, skipping creation")
        return
    log("Unkown object type", g_type, ", skipping initialization")


def add_basic_shape(g_name, g_type, g_pos, g_speed, g_mats, geometry, objects, base_dir=None):
    """scene_parser.py:212-258 (textures: Image.open of the path, scale default 1.0)."""
    if g_type == "sphere":
        g_radius = geometry["radius"]
        objects.append(geom.Sphere(g_name, g_type, g_mats, g_pos, g_radius, g_speed))
    elif g_type == "plane":
        g_normal = populateVec(geometry["normal"])
        plane = geom.Plane(g_name, g_type, g_mats, g_pos, g_normal, g_speed)
        if "texture" in geometry:
            plane.texture = geom.open_texture(geometry["texture"], base_dir)
            plane.texture_scale = get_or(geometry, "texture_scale", 1.0)
        objects.append(plane)
    elif g_type == "box":
        try:
            g_size = populateVec(geometry["size"])
            box = geom.AABB(g_name, g_type, g_mats, g_pos, g_size, g_speed)
        except KeyError:
            box = geom.AABB(g_name, g_type, g_mats, g_pos, [0, 0, 0], g_speed)
            box.minpos = geom.F.vec3(populateVec(geometry["min"]))
            box.maxpos = geom.F.vec3(populateVec(geometry["max"]))
        if "texture" in geometry:
            box.texture = geom.open_texture(geometry["texture"], base_dir)
        objects.append(box)
    elif g_type == "mesh":
        g_path = geom.resolve_path(geometry["filepath"], base_dir)
        g_scale = geometry["scale"]
        g_flat_shaded = get_or(geometry, "flat_shaded", False)
        objects.append(geom.Mesh(g_name, g_type, g_mats, g_pos, g_scale, g_path, g_flat_shaded, g_speed))
    else:
        return False
    return True


def traverse_children(node, children, materials, rootNames, roots, speed, base_dir=None, log=print):
    """scene_parser.py:261-285: a child's speed is the root's speed plus its own (fp32);
    nested nodes pass the ROOT's speed on to their own children (:283)."""
    for geometry in children:
        g_name = geometry["name"]
        g_type = geometry["type"]
        g_pos = populateVec(get_or(geometry, "position", [0, 0, 0]))
        g_mats = associate_material(materials, get_or(geometry, "materials", []))
        if speed is None:
            g_speed = None
        else:
            g_speed = geom.F.vec3(speed) + geom.F.vec3(populateVec(get_or(geometry, "speed", [0, 0, 0])))
        if add_basic_shape(g_name, g_type, g_pos, g_speed, g_mats, geometry, node.children, base_dir):
            continue
        elif g_type == "node":
            g_r = populateVec(get_or(geometry, "rotation", [0, 0, 0]))
            g_s = populateVec(get_or(geometry, "scale", [1, 1, 1]))
            g_hierarchy_type = get_or(geometry, "hierarchy_type", "union")
            inner = geom.Hierarchy(g_name, g_type, g_mats, g_hierarchy_type, g_pos, g_r, g_s, g_speed)
            node.children.append(inner)
            traverse_children(inner, geometry["children"], materials, rootNames, roots, speed, base_dir, log)
        else:
            parse_geometry(geometry, node.children, rootNames, roots, materials, base_dir, log)


def associate_material(mats, ids):
    """scene_parser.py:288-294."""
    return [mat for i in ids for mat in mats if i == mat.ID]
