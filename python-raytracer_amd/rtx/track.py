"""Edit tracking of the scene description (objects, materials, lights, ambient).

The reference reads every object, material and light attribute on every render
(provided/scene.py:86-88, :148, :161-164), so an edit between two renders shows up in the
second. This package uploads the scene once (rtx_scene_create); to keep the reference's
behaviour without flattening the scene on every frame, its own description classes
(rtx.geometry, rtx.helperclasses Material / Light, the Scene's lists) report every change:

- an attribute assignment on a ``Tracked`` object,
- an in-place write into one of its arrays (``sphere.center[0] = 2``, ``mat.diffuse *= 0.5``,
  a slice of ``mesh.verts``), kept as ``TArray``,
- a change of one of its lists (``obj.materials.append``, ``scene.objects.pop``) when it is
  a ``TList`` (the lists this package's constructors and parser create),

counts one process-wide epoch up. ``rtx.Scene`` compares the epoch per render (one integer
compare); when it moved, the scene is flattened again and re-uploaded if its records
differ (a digest of the descriptor bytes). Scenes whose objects are not all tracked -- the
reference's own objects bound by ``Scene.from_reference``, plain lists handed to a
constructor, or an attribute of another mutable type such as a PyGLM vector -- are
flattened and compared on every render instead. Writes that bypass both hooks
(``np.copyto``, ``ndarray.fill``, a ``.view(np.ndarray)``, another reference to an array's
memory, the pixels of a texture image) are not seen: call ``Scene.invalidate()`` after them.
"""
import numpy as np

_EPOCH = [0]


def epoch():
    """The process-wide edit counter."""
    return _EPOCH[0]


def bump():
    _EPOCH[0] += 1


class TArray(np.ndarray):
    """An array attribute of a tracked object: item assignment (also through a view) and
    ufuncs writing into it (``a += b``, ``np.add(x, y, out=a)``) count the epoch up.
    Arithmetic on it returns plain arrays."""

    def __setitem__(self, key, value):
        super().__setitem__(key, value)
        bump()

    def __array_ufunc__(self, ufunc, method, *inputs, out=None, **kwargs):
        plain = [x.view(np.ndarray) if isinstance(x, TArray) else x for x in inputs]
        if out is None:
            r = getattr(ufunc, method)(*plain, **kwargs)
            if method == "at" and isinstance(inputs[0], TArray):  # np.add.at(a, idx, v): in place
                bump()
            return r
        kwargs["out"] = tuple(o.view(np.ndarray) if isinstance(o, TArray) else o for o in out)
        getattr(ufunc, method)(*plain, **kwargs)
        if any(isinstance(o, TArray) for o in out):
            bump()
        return out[0] if len(out) == 1 else out


class TList(list):
    """A list attribute of a tracked object (or a Scene's objects / materials / lights):
    every in-place change counts the epoch up. It compares equal to a plain list."""


def _tracked_list_method(name):
    base = getattr(list, name)

    def method(self, *args, **kwargs):
        r = base(self, *args, **kwargs)
        bump()
        return self if name in ("__iadd__", "__imul__") else r
    method.__name__ = name
    return method


for _m in ("__setitem__", "__delitem__", "__iadd__", "__imul__", "append", "extend", "insert", "pop", "remove",
           "clear", "sort", "reverse"):
    setattr(TList, _m, _tracked_list_method(_m))

# values that cannot change in place (or are tracked themselves)
_IMMUTABLE = (type(None), bool, int, float, complex, str, bytes, tuple, frozenset, np.generic)


def _is_image(v):
    return type(v).__module__.startswith("PIL.")


class Tracked:
    """Base of the tracked description classes: every attribute assignment counts the epoch
    up, and arrays are kept as TArray views (the same memory). A list that is not a TList,
    or a value of another mutable type (a PyGLM vector), is kept as given -- the caller may
    still hold and change it, as the reference's objects share them -- and marks the
    object untracked while it is assigned: its scenes are then compared per render. The
    constructors of this package create TLists for the lists they own. Attributes named in
    ``_NOT_RECORDS`` (``scene``: the back-reference set_scene stores) are not part of the
    records and are neither wrapped nor counted."""

    _NOT_RECORDS = ("scene",)

    def __setattr__(self, name, value):
        if name.startswith("_") or name in self._NOT_RECORDS:
            object.__setattr__(self, name, value)
            return
        if isinstance(value, np.ndarray) and not isinstance(value, TArray):
            value = value.view(TArray)
        plain = not (isinstance(value, (TArray, TList, Tracked) + _IMMUTABLE) or _is_image(value))
        loose = self.__dict__.get("_loose")
        if plain:
            if loose is None:
                loose = set()
                object.__setattr__(self, "_loose", loose)
            loose.add(name)
        elif loose:
            loose.discard(name)
        object.__setattr__(self, name, value)
        bump()

    def __deepcopy__(self, memo):
        # (the copy's state is restored without __setattr__; count it as an edit). The
        # scene back-reference is shared, not copied: the copy belongs to the same scene.
        import copy
        cls = type(self)
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            object.__setattr__(new, k, v if k in self._NOT_RECORDS else copy.deepcopy(v, memo))
        bump()
        return new


def is_tracked(x):
    return isinstance(x, Tracked) and not x.__dict__.get("_loose")


def scene_tracked(objects, materials, lights, ambient):
    """True when every record the scene flattens is reported by the hooks above: the
    lists are TLists and every object (hierarchies' children included), material, light
    and bounding volume is a tracked object."""
    if not (isinstance(objects, TList) and isinstance(materials, TList) and isinstance(lights, TList)
            and isinstance(ambient, TArray)):
        return False
    stack = list(objects)
    while stack:
        g = stack.pop()
        if not is_tracked(g):
            return False
        mats = g.__dict__.get("materials")
        if mats is not None and not (isinstance(mats, TList) and all(is_tracked(m) for m in mats)):
            return False
        bv = g.__dict__.get("bounding_volume")
        if bv is not None and not is_tracked(bv):
            return False
        children = g.__dict__.get("children")
        if children is not None:
            if not isinstance(children, TList):
                return False
            stack.extend(children)
    return all(is_tracked(m) for m in materials) and all(is_tracked(L) for L in lights)
