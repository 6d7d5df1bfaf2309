"""Scene catalog — the reference's scene builders (src/main.rs) restated.

Each builder returns a ``Scene`` (spec, camera arguments, SampleSettings) with the
reference's values; ``config(name)`` gives the BASELINE.json configurations C1..C5
(SURVEY.md §8d).  The reference draws scene randomness from an unseeded fastrand;
here it is one wyrand stream seeded with SCENE_SEED ("grayshif"), consumed in
main.rs's draw order, so every run builds the same world.
"""
import math
import struct
from dataclasses import dataclass

from . import assets
from .scene import SceneBuilder, camera_spec, fixed_spp, sample_settings

SCENE_SEED = 0x6772617973686966  # b"grayshif"
_M64 = (1 << 64) - 1


class Wyrand:
    """fastrand 2.1.1 ``Rng`` (wyrand): gen_u64 and f64, as restated in oracle.cpp."""

    C0, C1 = 0x2D358DCCAA6C78A5, 0x8BB84B93962EACC9

    def __init__(self, seed):
        self.state = seed & _M64

    def u64(self):
        s = (self.state + self.C0) & _M64
        self.state = s
        t = s * (s ^ self.C1)
        return (t & _M64) ^ (t >> 64)

    def f64(self):
        bits = 0x3FF0000000000000 | (self.u64() >> 12)
        return struct.unpack("<d", struct.pack("<Q", bits))[0] - 1.0

    def random_f64(self, lo, hi):  # util.rs:5-7
        return self.f64() * (hi - lo) + lo

    def random_vector(self, lo, hi):  # util.rs:9-16 (x, y, z drawn in order)
        x = self.random_f64(lo, hi)
        y = self.random_f64(lo, hi)
        z = self.random_f64(lo, hi)
        return (x, y, z)


@dataclass
class Scene:
    name: str
    spec: object  # scene.SceneSpec
    camera: object  # gs_camera_spec
    settings: object  # gs_sample_settings

    @property
    def width(self):
        return self.camera.image_width

    @property
    def height(self):
        return int(self.camera.image_width / self.camera.aspect_ratio)


def _camera(aspect, width, depth, vfov, frm, at, vup, defocus, focus):
    return camera_spec(aspect, width, depth, vfov, frm, at, vup, defocus, focus)


def _hdri_background(b, rotation):
    b.background_hdri(assets.airport_hdr_f32(), rotation)


# --------------------------------------------------------------------- scenes
def _bouncing_content(b, grid, rng):
    """The world of main.rs:61-152 (ground, grid of small spheres, three big ones)."""
    ground = b.lambertian_texture(b.checkered_from_colors(0.32, (0.2, 0.3, 0.1), (0.9, 0.9, 0.9)))
    b.add(b.sphere((0.0, -1000.0, 0.0), 1000.0, ground))
    for a in range(-grid, grid):
        for bb in range(-grid, grid):
            cx = a + 0.9 * rng.f64()
            cz = bb + 0.9 * rng.f64()
            center = (float(cx), 0.2, float(cz))
            dx, dy, dz = center[0] - 4.0, center[1] - 0.2, center[2] - 0.0
            if math.sqrt(dx * dx + dy * dy + dz * dz) > 0.9:
                choice = rng.f64()
                if choice < 0.8:
                    v1 = rng.random_vector(0.0, 1.0)
                    v2 = rng.random_vector(0.0, 1.0)
                    mat = b.lambertian((v1[0] * v2[0], v1[1] * v2[1], v1[2] * v2[2]))
                elif choice < 0.95:
                    albedo = rng.random_vector(0.5, 1.0)
                    fuzz = rng.random_f64(0.0, 0.5)
                    mat = b.metal(albedo, fuzz)
                else:
                    mat = b.dielectric(1.5)
                rng.f64()  # center_end (main.rs:110): drawn, unused
                b.add(b.sphere(center, 0.2, mat))
    b.add(b.sphere((4.0, 1.0, 0.0), 1.0, b.metal((0.7, 0.6, 0.5), 0.0)))
    b.add(b.sphere((0.0, 1.0, 0.0), 1.0, b.dielectric(1.5)))
    b.add(b.sphere((-4.0, 1.0, 0.0), 1.0, b.metal((0.7, 0.6, 0.5), 0.0)))


def bouncing_spheres(grid=11, width=600, settings=None):
    """main.rs:61-167 with the grid half-width as a parameter (C4 uses 50)."""
    b = SceneBuilder()
    _bouncing_content(b, grid, Wyrand(SCENE_SEED))
    _hdri_background(b, (0.0, -90.0, 90.0))  # "degrees" passed as radians (main.rs:159)
    cam = _camera(16.0 / 9.0, width, 50, 20.0, (13.0, 2.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.6, 10.0)
    return Scene("bouncing_spheres_%d" % grid, b.build(), cam, settings or sample_settings(0.95, 0.05, 64, 200))


def checkered_spheres(width=400, settings=None):  # main.rs:169-215
    b = SceneBuilder()
    m = b.lambertian_texture(b.checkered_from_colors(0.32, (0.2, 0.3, 0.1), (0.9, 0.9, 0.9)))
    b.add(b.sphere((0.0, -10.0, 0.0), 10.0, m))
    b.add(b.sphere((0.0, 10.0, 0.0), 10.0, m))
    b.background_solid((0.7, 0.8, 1.0))
    cam = _camera(16.0 / 9.0, width, 50, 20.0, (13.0, 2.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    return Scene("checkered_spheres", b.build(), cam, settings or sample_settings(0.95, 0.25, 32, 1000))


def earth(width=400, settings=None, hdri=False):
    """main.rs:217-253.  hdri=True swaps the solid sky for hdri()'s airport.hdr
    background (rotation (pi/2, pi, 0), main.rs:824-827): BASELINE configs C1/C2."""
    b = SceneBuilder()
    tex = b.image_texture(b.image(assets.earthmap_rgb8()))
    b.add(b.sphere((0.0, 0.0, 0.0), 2.0, b.lambertian_texture(tex)))
    if hdri:
        _hdri_background(b, (math.pi / 2.0, math.pi, 0.0))
    else:
        b.background_solid((0.7, 0.8, 1.0))
    cam = _camera(16.0 / 9.0, width, 50, 20.0, (0.0, 0.0, 12.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    return Scene("earth_hdr" if hdri else "earth", b.build(), cam, settings or sample_settings(0.95, 0.25, 32, 1000))


def perlin_spheres(width=400, settings=None):  # main.rs:255-297
    b = SceneBuilder()
    m = b.lambertian_texture(b.noise(4.0))
    b.add(b.sphere((0.0, -1000.0, 0.0), 1000.0, m))
    b.add(b.sphere((0.0, 2.0, 0.0), 2.0, m))
    b.background_solid((0.7, 0.8, 1.0))
    cam = _camera(16.0 / 9.0, width, 50, 20.0, (13.0, 2.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    return Scene("perlin_spheres", b.build(), cam, settings or sample_settings(0.95, 0.25, 32, 1000))


def simple_light(width=1000, settings=None):  # main.rs:366-419
    b = SceneBuilder()
    m = b.lambertian_texture(b.noise(4.0))
    b.add(b.sphere((0.0, -1000.0, 0.0), 1000.0, m))
    b.add(b.sphere((0.0, 2.0, 0.0), 2.0, m))
    b.add(b.quad((3.0, 1.0, -2.0), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), b.diffuse_light((4.0, 4.0, 4.0))))
    b.background_solid((0.0, 0.0, 0.0))
    cam = _camera(16.0 / 9.0, width, 50, 20.0, (26.0, 3.0, 6.0), (0.0, 2.0, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    return Scene("simple_light", b.build(), cam, settings or sample_settings(0.95, 0.25, 32, 1000))


def final_scene(width=800, settings=None, max_depth=40, boxes_per_side=20, n_balls=1000):
    """main.rs:626-790 (SCENE 9: width 800, depth 40; SCENE 8: 400, 50).  Everything the
    reference uses: a BVH of 400 cubes inside the world BVH, a light quad, a moving
    sphere, glass / metal / earth / noise spheres, two media (a foggy glass sphere and a
    world fog), and a BVH of 1000 balls under Translate(RotateY).  The scene draws come
    from one wyrand stream in main.rs's order (box heights, then ball centres)."""
    rng = Wyrand(SCENE_SEED)
    b = SceneBuilder()
    ground = b.lambertian((0.48, 0.83, 0.53))
    boxes = []
    for i in range(boxes_per_side):
        for j in range(boxes_per_side):
            w = 100.0
            x0 = -1000.0 + i * w
            z0 = -1000.0 + j * w
            y1 = rng.random_f64(1.0, 101.0)
            boxes.append(b.cube((x0, 0.0, z0), (x0 + w, y1, z0 + w), ground))
    b.add(b.bvh(boxes))
    b.add(b.quad((123.0, 554.0, 147.0), (300.0, 0.0, 0.0), (0.0, 0.0, 265.0), b.diffuse_light((7.0, 7.0, 7.0))))
    c1 = (400.0, 400.0, 200.0)
    b.add(b.moving_sphere(c1, (c1[0] + 30.0, c1[1], c1[2]), 50.0, b.lambertian((0.7, 0.3, 0.1))))
    b.add(b.sphere((260.0, 150.0, 45.0), 50.0, b.dielectric(1.5)))
    b.add(b.sphere((0.0, 150.0, 145.0), 50.0, b.metal((0.8, 0.8, 0.9), 1.0)))
    b.add(b.sphere((400.0, 200.0, 400.0), 100.0, b.lambertian_texture(b.image_texture(b.image(assets.earthmap_rgb8())))))
    b.add(b.sphere((220.0, 280.0, 300.0), 80.0, b.lambertian_texture(b.noise(0.2))))
    fog = b.dielectric(1.5)
    b.add(b.medium(b.sphere((360.0, 150.0, 145.0), 70.0, fog), 0.2, b.lambertian((0.2, 0.4, 0.9))))
    b.add(b.medium(b.sphere((0.0, 0.0, 0.0), 5000.0, fog), 0.0001, b.lambertian((1.0, 1.0, 1.0))))
    white = b.lambertian((0.73, 0.73, 0.73))
    balls = [b.sphere(rng.random_vector(0.0, 165.0), 10.0, white) for _ in range(n_balls)]
    b.add(b.translate(b.rotate_y(b.bvh(balls), 15.0), (-100.0, 270.0, 395.0)))
    b.background_solid((0.0, 0.0, 0.0))
    cam = _camera(1.0, width, max_depth, 40.0, (478.0, 278.0, -600.0), (278.0, 278.0, 0.0), (0.0, 1.0, 0.0), 0.0,
                  10.0)
    return Scene("final_scene", b.build(), cam, settings or sample_settings(0.95, 0.25, 32, 1000))


def quads(width=400, settings=None):  # main.rs:299-364
    b = SceneBuilder()
    b.add(b.quad((-3.0, -2.0, 5.0), (0.0, 0.0, -4.0), (0.0, 4.0, 0.0), b.lambertian((1.0, 0.2, 0.2))))
    b.add(b.quad((-2.0, -2.0, 0.0), (4.0, 0.0, 0.0), (0.0, 4.0, 0.0), b.lambertian((0.2, 1.0, 0.2))))
    b.add(b.quad((3.0, -2.0, 1.0), (0.0, 0.0, 4.0), (0.0, 4.0, 0.0), b.lambertian((0.2, 0.2, 1.0))))
    b.add(b.quad((-2.0, 3.0, 1.0), (4.0, 0.0, 0.0), (0.0, 0.0, 4.0), b.lambertian((1.0, 0.5, 0.0))))
    b.add(b.quad((-2.0, -3.0, 5.0), (4.0, 0.0, 0.0), (0.0, 0.0, -4.0), b.lambertian((0.2, 0.8, 0.8))))
    b.background_solid((0.7, 0.8, 1.0))
    cam = _camera(1.0, width, 50, 80.0, (0.0, 0.0, 9.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    return Scene("quads", b.build(), cam, settings or sample_settings(0.95, 0.25, 32, 1000))


def _cornell_walls(b, light_q, light_u, light_v, light_rgb):
    red = b.lambertian((0.65, 0.05, 0.05))
    white = b.lambertian((0.73, 0.73, 0.73))
    green = b.lambertian((0.12, 0.45, 0.15))
    light = b.diffuse_light(light_rgb)
    b.add(b.quad(light_q, light_u, light_v, light))
    b.add(b.quad((555.0, 0.0, 0.0), (0.0, 555.0, 0.0), (0.0, 0.0, 555.0), green))
    b.add(b.quad((0.0, 0.0, 0.0), (0.0, 555.0, 0.0), (0.0, 0.0, 555.0), red))
    b.add(b.quad((0.0, 0.0, 0.0), (555.0, 0.0, 0.0), (0.0, 0.0, 555.0), white))
    b.add(b.quad((555.0, 555.0, 555.0), (-555.0, 0.0, 0.0), (0.0, 0.0, -555.0), white))
    b.add(b.quad((0.0, 0.0, 555.0), (555.0, 0.0, 0.0), (0.0, 555.0, 0.0), white))
    return white


def cornell_box(width=600, settings=None):  # main.rs:421-517
    b = SceneBuilder()
    white = _cornell_walls(b, (343.0, 554.0, 332.0), (-130.0, 0.0, 0.0), (0.0, 0.0, -105.0), (15.0, 15.0, 15.0))
    box1 = b.cube((0.0, 0.0, 0.0), (165.0, 330.0, 165.0), white)
    b.add(b.translate(b.rotate_y(box1, 15.0), (265.0, 0.0, 295.0)))
    box2 = b.cube((0.0, 0.0, 0.0), (165.0, 165.0, 165.0), white)
    b.add(b.translate(b.rotate_y(box2, -18.0), (130.0, 0.0, 65.0)))
    b.background_solid((0.0, 0.0, 0.0))
    cam = _camera(1.0, width, 50, 40.0, (278.0, 278.0, -800.0), (278.0, 278.0, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    return Scene("cornell_box", b.build(), cam, settings or sample_settings(0.95, 0.5, 32, 1000))


def cornell_smoke(width=600, settings=None):  # main.rs:519-624
    b = SceneBuilder()
    white = _cornell_walls(b, (113.0, 554.0, 127.0), (330.0, 0.0, 0.0), (0.0, 0.0, 305.0), (7.0, 7.0, 7.0))
    box1 = b.cube((0.0, 0.0, 0.0), (165.0, 330.0, 165.0), white)
    b.add(b.medium_isotropic(b.translate(b.rotate_y(box1, 15.0), (265.0, 0.0, 295.0)), 0.01, (0.0, 0.0, 0.0)))
    box2 = b.cube((0.0, 0.0, 0.0), (165.0, 165.0, 165.0), white)
    b.add(b.medium_isotropic(b.translate(b.rotate_y(box2, -18.0), (130.0, 0.0, 65.0)), 0.01, (1.0, 1.0, 1.0)))
    b.background_solid((0.0, 0.0, 0.0))
    cam = _camera(1.0, width, 50, 40.0, (278.0, 278.0, -800.0), (278.0, 278.0, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    return Scene("cornell_smoke", b.build(), cam, settings or sample_settings(0.95, 0.25, 32, 1000))


def hdri(width=600, settings=None):  # main.rs:792-834 — the literal default (SCENE = 11)
    b = SceneBuilder()
    b.add(b.sphere((4.0, 1.0, 0.0), 1.0, b.metal((0.7, 0.6, 0.5), 0.0)))
    _hdri_background(b, (math.pi / 2.0, math.pi, 0.0))
    cam = _camera(16.0 / 9.0, width, 50, 20.0, (13.0, 2.0, 5.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.6, 10.0)
    return Scene("hdri", b.build(), cam, settings or sample_settings(0.95, 0.05, 64, 200))


def triangles(width=400, settings=None):  # main.rs:836-887
    b = SceneBuilder()
    b.add(b.triangle((-2.0, 2.0, 0.0), (-2.0, -2.0, 0.0), (-2.0, -2.0, 4.0), b.lambertian((1.0, 0.2, 0.2))))
    b.add(b.triangle((-2.0, 2.0, 0.0), (2.0, -2.0, 0.0), (-2.0, -2.0, 0.0), b.lambertian((0.2, 1.0, 0.2))))
    b.add(b.triangle((-2.0, -2.0, 4.0), (-2.0, -2.0, 0.0), (2.0, -2.0, 0.0), b.lambertian((1.0, 0.5, 0.0))))
    b.background_solid((0.7, 0.8, 1.0))
    cam = _camera(1.0, width, 50, 80.0, (0.0, 0.0, 9.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.0, 10.0)
    return Scene("triangles", b.build(), cam, settings or sample_settings(0.95, 0.25, 32, 1000))


def mixed(width=3840, settings=None):
    """C5: the bouncing-spheres generator at grid [-11, 11) plus the
    earthmap sphere, a Cornell-style light and wall, RotateY/Translate cubes, a
    triangle fan and a moving sphere, under the airport.hdr sky.  Defined here
    (the reference has no such scene); every element is a reference type."""
    b = SceneBuilder()
    _bouncing_content(b, 11, Wyrand(SCENE_SEED))
    # earth sphere (ImageTexture)
    b.add(b.sphere((-8.0, 2.0, 2.5), 2.0, b.lambertian_texture(b.image_texture(b.image(assets.earthmap_rgb8())))))
    # Cornell-style light panel and back wall (quads)
    b.add(b.quad((-6.0, 6.0, -4.0), (4.0, 0.0, 0.0), (0.0, 0.0, 3.0), b.diffuse_light((6.0, 6.0, 6.0))))
    b.add(b.quad((-12.0, 0.0, -6.0), (10.0, 0.0, 0.0), (0.0, 5.0, 0.0), b.lambertian((0.65, 0.05, 0.05))))
    # RotateY / Translate cubes
    white = b.lambertian((0.73, 0.73, 0.73))
    b.add(b.translate(b.rotate_y(b.cube((0.0, 0.0, 0.0), (1.0, 2.0, 1.0), white), 15.0), (6.0, 0.0, -3.0)))
    b.add(b.translate(b.rotate_y(b.cube((0.0, 0.0, 0.0), (1.2, 1.2, 1.2), b.metal((0.8, 0.8, 0.9), 0.1)), -18.0),
                      (7.0, 0.0, 2.0)))
    # triangle fan
    fan_mat = b.lambertian((1.0, 0.5, 0.0))
    c = (2.0, 3.5, -5.0)
    for k in range(6):
        a0 = 2.0 * math.pi * k / 6.0
        a1 = 2.0 * math.pi * (k + 1) / 6.0
        p0 = (c[0] + 1.5 * math.cos(a0), c[1] + 1.5 * math.sin(a0), c[2])
        p1 = (c[0] + 1.5 * math.cos(a1), c[1] + 1.5 * math.sin(a1), c[2])
        b.add(b.triangle(c, p1, p0, fan_mat))
    # moving sphere
    b.add(b.moving_sphere((-2.0, 0.5, 3.0), (-2.0, 0.9, 3.0), 0.5, b.lambertian((0.7, 0.3, 0.1))))
    _hdri_background(b, (0.0, -90.0, 90.0))
    cam = _camera(16.0 / 9.0, width, 50, 30.0, (13.0, 2.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.6, 10.0)
    return Scene("mixed", b.build(), cam, settings or sample_settings(0.95, 0.05, 64, 200))


SCENES = {
    "bouncing_spheres": bouncing_spheres,
    "checkered_spheres": checkered_spheres,
    "earth": earth,
    "earth_hdr": lambda width=400, settings=None: earth(width, settings, hdri=True),
    "quads": quads,
    "cornell_box": cornell_box,
    "cornell_smoke": cornell_smoke,
    "hdri": hdri,
    "triangles": triangles,
    "mixed": mixed,
    "perlin_spheres": perlin_spheres,
    "simple_light": simple_light,
    "final_scene": final_scene,
}

# BASELINE.json configs: (builder, kwargs, width, spp).  spp None: the
# scene's own adaptive SampleSettings, as main.rs renders every scene -- A1 the literal
# default scene hdri() (main.rs:811-815: confidence 0.95, tolerance 0.05, batch 64, max 200)
# at 1080p, A2 cornell_box (main.rs:497-501: 0.95, 0.5, 32, 1000) at 1024 x 1024.
CONFIGS = {
    "C1": ("earth_hdr", {}, 400, 100),
    "C2": ("earth_hdr", {}, 1920, 256),
    "C3": ("cornell_box", {}, 1024, 1024),
    "C4": ("bouncing_spheres", {"grid": 50}, 1920, 512),
    "C5": ("mixed", {}, 3840, 4096),
    "A1": ("hdri", {}, 1920, None),
    "A2": ("cornell_box", {}, 1024, None),
}


def config(name, width=None, spp=None):
    """A BASELINE config; width/spp overrides give the small parity-test versions (spp on an
    adaptive config replaces its settings by fixed spp).  A reference scene's name (SCENES)
    gives that scene at fixed spp (default 400 px, 64 spp)."""
    if name not in CONFIGS and name in SCENES:
        return SCENES[name](width=width or 400, settings=fixed_spp(spp or 64))
    scene, kw, w, s = CONFIGS[name]
    if s is None and spp is None:
        return SCENES[scene](width=width or w, **kw)  # the scene's own adaptive settings
    return SCENES[scene](width=width or w, settings=fixed_spp(spp or s), **kw)
