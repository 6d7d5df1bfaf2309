"""A third, independent restatement of the world-building arithmetic, checked against the
product host (grayshift_amd/csrc/host/world.cpp, which flattens for the device).

The product host and the CPU oracle (oracle/oracle.cpp) were transcribed by the same
hand and share text (RotateY's box, Quad::cube, the BVH build), so a transcription
error could sit in both and pass every oracle test.  This file restates those pieces
from the reference afresh, in Python floats (IEEE f64, no FMA), in a different shape
(plain tuples and functions, no classes), and compares the product's flattened world
with it exactly: every BVH node's f64 box in pre-order, the left/right structure, and
every primitive record (sphere, moving sphere, quad with its derived w / normal / d,
triangle with its normal, lists, Translate / RotateY transforms, media).

Reference (file:line): AABB.rs:24-56 (from_corners, pad), :115-128 (longest_axis,
pad_to_minimums); interval.rs:10-44; BVH.rs:18-65 (construct_tree); sphere.rs:21-49;
quad.rs:25-38, :54-80 (cube); plane.rs:15-18; triangle.rs:20-28; hittable.rs:62-66
(HittableList::add), :100-104 (Translate::new), :135-175 (RotateY::new);
volume.rs:17-21, :65-67; util.rs:62-64 (deg_to_rad); vec3.rs:19-43.
"""
import ctypes as C
import math

import pytest

from grayshift_amd import _native as N
from grayshift_amd import scenes
from grayshift_amd.renderer import HostScene

F64_MAX = 1.7976931348623157e308
EMPTY = ((F64_MAX, -F64_MAX),) * 3  # Interval::EMPTY per axis (interval.rs:10)


# ---- vec3.rs / interval.rs / AABB.rs, as functions on tuples
def vsub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def vadd(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def vdot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def vcross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def vdiv(a, s):
    return (a[0] / s, a[1] / s, a[2] / s)


def expand(iv, delta):  # interval.rs:41-44
    pad = delta / 2.0
    return (iv[0] - pad, iv[1] + pad)


def corners(a, b):  # AABB.rs:24-47 with pad_to_minimums (:123-128)
    box = []
    for k in range(3):
        iv = (a[k], b[k]) if a[k] <= b[k] else (b[k], a[k])
        if iv[1] - iv[0] < 0.0001:
            iv = expand(iv, 0.0001)
        box.append(iv)
    return tuple(box)


def union(p, q):  # AABB::from_AABB_pair / Interval::from_interval_pair
    return tuple((p[k][0] if p[k][0] <= q[k][0] else q[k][0], p[k][1] if p[k][1] >= q[k][1] else q[k][1])
                 for k in range(3))


def longest(b):  # AABB.rs:115-121
    sx, sy, sz = (b[k][1] - b[k][0] for k in range(3))
    if sx > sy:
        return 0 if sx > sz else 2
    return 1 if sy > sz else 2


# ---- the objects of a scene spec, as (box, tree) pairs; tree = what the flat scene holds
def build(spec, idx):
    o = spec.objects[idx]
    p = list(o.p)
    kids = lambda: [build(spec, spec.children[o.first + i]) for i in range(o.count)]
    if o.kind == N.GS_OBJ_SPHERE:  # sphere.rs:21-33
        c, r = tuple(p[:3]), p[3]
        rv = (r, r, r)
        return corners(vsub(c, rv), vadd(c, rv)), ("sphere", c, r)
    if o.kind == N.GS_OBJ_MOVING_SPHERE:  # sphere.rs:35-49
        c1, c2, r = tuple(p[:3]), tuple(p[3:6]), p[6]
        rv = (r, r, r)
        box = union(corners(vsub(c1, rv), vadd(c1, rv)), corners(vsub(c2, rv), vadd(c2, rv)))
        return box, ("msphere", c1, vsub(c2, c1), r)
    if o.kind == N.GS_OBJ_QUAD:
        return quad(tuple(p[:3]), tuple(p[3:6]), tuple(p[6:9]))
    if o.kind == N.GS_OBJ_TRIANGLE:  # triangle.rs:20-28
        a, b, c = tuple(p[:3]), tuple(p[3:6]), tuple(p[6:9])
        return union(corners(a, b), corners(a, c)), ("tri", a, b, c, vcross(vsub(b, a), vsub(c, a)))
    if o.kind == N.GS_OBJ_CUBE:
        return hlist(cube(tuple(p[:3]), tuple(p[3:6])))
    if o.kind == N.GS_OBJ_LIST:
        return hlist(kids())
    if o.kind == N.GS_OBJ_BVH:
        return bvh(kids())
    if o.kind == N.GS_OBJ_TRANSLATE:  # hittable.rs:100-104: bbox + offset
        box, tree = build(spec, o.first)
        off = tuple(p[:3])
        return tuple((box[k][0] + off[k], box[k][1] + off[k]) for k in range(3)), ("translate", off, tree)
    if o.kind == N.GS_OBJ_ROTATE_Y:
        return rotate_y(build(spec, o.first), p[0])
    if o.kind == N.GS_OBJ_MEDIUM:  # volume.rs:17-21, :65-67
        box, tree = build(spec, o.first)
        return box, ("medium", -1.0 / p[0], tree)
    raise AssertionError("object kind %d" % o.kind)


def quad(q, u, v):  # quad.rs:25-38, plane.rs:15-18
    box = union(corners(q, vadd(vadd(q, u), v)), corners(vadd(q, u), vadd(q, v)))
    n = vcross(u, v)
    normal = vdiv(n, math.sqrt(vdot(n, n)))
    w = vdiv(n, vdot(n, n))
    return box, ("quad", q, u, v, w, normal, vdot(normal, q))


def cube(a, b):  # quad.rs:54-80 (f64::min / max, no NaNs here)
    mn = tuple(min(a[k], b[k]) for k in range(3))
    mx = tuple(max(a[k], b[k]) for k in range(3))
    dx, dy, dz = (mx[0] - mn[0], 0.0, 0.0), (0.0, mx[1] - mn[1], 0.0), (0.0, 0.0, mx[2] - mn[2])
    neg = lambda t: (-t[0], -t[1], -t[2])
    return [quad((mn[0], mn[1], mx[2]), dx, dy), quad((mx[0], mn[1], mx[2]), neg(dz), dy),
            quad((mx[0], mn[1], mn[2]), neg(dx), dy), quad((mn[0], mn[1], mn[2]), dz, dy),
            quad((mn[0], mx[1], mx[2]), dx, neg(dz)), quad((mn[0], mn[1], mn[2]), dx, dz)]


def hlist(members):  # hittable.rs:62-66: bbox grown from EMPTY member by member
    box = EMPTY
    for b, _ in members:
        box = union(box, b)
    return box, ("list", [t for _, t in members])


def rotate_y(child, angle):  # hittable.rs:135-175, util.rs:62-64
    box, tree = child
    rad = angle / 180.0 * math.pi
    s, c = math.sin(rad), math.cos(rad)
    mn, mx = [F64_MAX] * 3, [-F64_MAX] * 3
    for i in range(2):
        for j in range(2):
            for k in range(2):
                x = float(i) * box[0][1] + float(1 - i) * box[0][0]
                y = float(j) * box[1][1] + float(1 - j) * box[1][0]
                z = float(k) * box[2][1] + float(1 - k) * box[2][0]
                nx, nz = c * x + s * z, -s * x + c * z
                mn = [min(mn[0], nx), min(mn[1], y), min(mn[2], nz)]
                mx = [max(mx[0], nx), max(mx[1], y), max(mx[2], nz)]
    return corners(tuple(mn), tuple(mx)), ("rotate", s, c, tree)


def bvh(objs):  # BVH.rs:18-65
    if len(objs) == 1:
        return objs[0][0], ("node", objs[0][0], objs[0][1], None)
    if len(objs) == 2:
        box = union(objs[0][0], objs[1][0])
        return box, ("node", box, objs[0][1], objs[1][1])
    box = EMPTY
    for b, _ in objs:
        box = union(box, b)
    axis = longest(box)
    objs = sorted(objs, key=lambda bt: bt[0][axis][0])  # stable, as Rust's sort_by
    mid = len(objs) // 2
    left, right = bvh(objs[:mid]), bvh(objs[mid:])
    return box, ("node", box, left[1], right[1])


# ---- the product's flattened world, read back into the same shape
def from_flat(f, ref):
    kind, i = ref >> 28, ref & 0x0FFFFFFF
    t3 = lambda a: (a[0], a[1], a[2])
    if kind == 1:
        n = f.nodes[i]
        box = tuple((n.min[k], n.max[k]) for k in range(3))
        return ("node", box, from_flat(f, n.left), None if n.right == 0 else from_flat(f, n.right))
    if kind == 2:
        s = f.spheres[i]
        return ("sphere", t3(s.center), s.radius)
    if kind == 3:
        s = f.mspheres[i]
        return ("msphere", t3(s.center_start), t3(s.center_path), s.radius)
    if kind == 4:
        q = f.quads[i]
        return ("quad", t3(q.q), t3(q.u), t3(q.v), t3(q.w), t3(q.normal), q.d)
    if kind == 5:
        t = f.triangles[i]
        return ("tri", t3(t.a), t3(t.b), t3(t.c), t3(t.normal))
    if kind == 6:
        l = f.lists[i]
        return ("list", [from_flat(f, f.list_refs[l.first + k]) for k in range(l.count)])
    if kind == 7:
        x = f.instances[i]
        if x.kind == 1:
            return ("translate", t3(x.p), from_flat(f, x.child))
        return ("rotate", x.p[0], x.p[1], from_flat(f, x.child))
    if kind == 8:
        m = f.media[i]
        return ("medium", m.density_neg_inv, from_flat(f, m.boundary))
    raise AssertionError("ref kind %d" % kind)


class _Rec(C.Structure):
    pass


def flat_arrays(h):
    """gs_flat_scene with typed record arrays (the ctypes mirror keeps void pointers)."""
    class NodeRec(C.Structure):
        _fields_ = [("min", C.c_double * 3), ("max", C.c_double * 3), ("left", C.c_uint32), ("right", C.c_uint32),
                    ("pad", C.c_uint32 * 2)]

    class SphereRec(C.Structure):
        _fields_ = [("center", C.c_double * 3), ("radius", C.c_double), ("material", C.c_uint32), ("pad", C.c_uint32)]

    class MSphereRec(C.Structure):
        _fields_ = [("center_start", C.c_double * 3), ("center_path", C.c_double * 3), ("radius", C.c_double),
                    ("material", C.c_uint32), ("pad", C.c_uint32)]

    class QuadRec(C.Structure):
        _fields_ = [(n, C.c_double * 3) for n in ("q", "u", "v", "w", "normal")] + [
            ("d", C.c_double), ("material", C.c_uint32), ("pad", C.c_uint32)]

    class TriRec(C.Structure):
        _fields_ = [(n, C.c_double * 3) for n in ("a", "b", "c", "normal")] + [("material", C.c_uint32),
                                                                                ("pad", C.c_uint32)]

    class ListRec(C.Structure):
        _fields_ = [("first", C.c_uint32), ("count", C.c_uint32)]

    class InstRec(C.Structure):
        _fields_ = [("kind", C.c_uint32), ("child", C.c_uint32), ("p", C.c_double * 3)]

    class MediumRec(C.Structure):
        _fields_ = [("boundary", C.c_uint32), ("material", C.c_uint32), ("density_neg_inv", C.c_double)]

    v = h.flat

    def arr(ptr, typ, n):
        return (typ * max(1, n)).from_address(ptr) if n else []

    out = _Rec()
    out.nodes = arr(v.nodes, NodeRec, v.n_nodes)
    out.spheres = arr(v.spheres, SphereRec, v.n_spheres)
    out.mspheres = arr(v.mspheres, MSphereRec, v.n_mspheres)
    out.quads = arr(v.quads, QuadRec, v.n_quads)
    out.triangles = arr(v.triangles, TriRec, v.n_triangles)
    out.lists = arr(v.lists, ListRec, v.n_lists)
    out.list_refs = arr(v.list_refs, C.c_uint32, v.n_list_refs)
    out.instances = arr(v.instances, InstRec, v.n_instances)
    out.media = arr(v.media, MediumRec, v.n_media)
    return out, v.root


def _scene(name):
    if name.startswith("C"):
        return scenes.config(name, width=32, spp=1)
    if name == "bouncing_11":
        return scenes.bouncing_spheres(grid=11, width=32)
    return scenes.SCENES[name](width=32)


@pytest.mark.parametrize("name", ["C3", "C4", "C5", "C1", "final_scene", "cornell_smoke", "triangles", "quads",
                                  "bouncing_11", "simple_light"])
def test_product_world_equals_independent_restatement(name):
    sc = _scene(name)
    spec = sc.spec
    world = [build(spec, spec.world[k]) for k in range(spec.n_world)]
    _, expect = bvh(world)  # main.rs: BVHNode::from_list(world)
    h = HostScene(spec)
    try:
        f, root = flat_arrays(h)
        got = from_flat(f, root)
    finally:
        h.close()
    assert got == expect  # exact: every f64 box coordinate, transform and record
