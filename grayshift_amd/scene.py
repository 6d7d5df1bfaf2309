"""Scene description builder — the Python face of include/grayshift_scene.h.

Mirrors the construction calls of the reference's scene builders (src/main.rs):
``Sphere::new_stationary``, ``Quad::new``, ``Quad::cube``, ``RotateY::new``,
``Translate::new``, ``Lambertian::from_color`` / ``from_texture``, ``Metal::new``,
``Dielectric::new``, ``DiffuseLight::from_color``, ``Isotropic::from_color``,
``ConstantMedium::new`` / ``from_isotropic_color``, ``CheckeredTexture::from_colors``,
``ImageTexture::new``, ``world.add``.  The result is a gs_scene_spec that both the
product host (C++) and the CPU oracle consume; neither side sees the other's world.
"""
import ctypes as C

import numpy as np

from . import _native as N


class SceneSpec:
    """Owns the ctypes arrays behind one gs_scene_spec (keep it alive while used)."""

    def __init__(self, objects, children, world, materials, textures, images, background, keep):
        self._keep = keep
        self.objects = (N.gs_object * max(1, len(objects)))(*objects)
        self.children = (C.c_int32 * max(1, len(children)))(*children)
        self.world = (C.c_int32 * max(1, len(world)))(*world)
        self.materials = (N.gs_material_spec * max(1, len(materials)))(*materials)
        self.textures = (N.gs_texture_spec * max(1, len(textures)))(*textures)
        self.images = (N.gs_image_spec * max(1, len(images)))(*images)
        s = N.gs_scene_spec()
        s.objects, s.n_objects = self.objects, len(objects)
        s.children, s.n_children = self.children, len(children)
        s.world, s.n_world = self.world, len(world)
        s.materials, s.n_materials = self.materials, len(materials)
        s.textures, s.n_textures = self.textures, len(textures)
        s.images, s.n_images = self.images, len(images)
        s.background = background
        self.spec = s
        self.n_world = len(world)

    def ptr(self):
        return C.byref(self.spec)


class SceneBuilder:
    def __init__(self):
        self._objects, self._children, self._world = [], [], []
        self._materials, self._textures, self._images = [], [], []
        self._keep = []
        self._bg = N.gs_background_spec()
        self.background_solid((0.0, 0.0, 0.0))

    # ------------------------------------------------------------- textures
    def solid(self, rgb):
        t = N.gs_texture_spec(kind=N.GS_TEX_SOLID, a=-1, b=-1)
        t.p[:] = [float(x) for x in rgb]
        self._textures.append(t)
        return len(self._textures) - 1

    def checkered(self, scale, even_tex, odd_tex):
        t = N.gs_texture_spec(kind=N.GS_TEX_CHECKERED, a=even_tex, b=odd_tex)
        t.p[0] = float(scale)
        self._textures.append(t)
        return len(self._textures) - 1

    def checkered_from_colors(self, scale, even_rgb, odd_rgb):  # texture.rs:49-55
        return self.checkered(scale, self.solid(even_rgb), self.solid(odd_rgb))

    def image(self, rgb8):
        a = np.ascontiguousarray(rgb8, dtype=np.uint8)
        if a.ndim != 3 or a.shape[2] != 3:
            raise ValueError("image must be HxWx3 uint8")
        self._keep.append(a)
        self._images.append(N.gs_image_spec(width=a.shape[1], height=a.shape[0], rgb8=a.ctypes.data))
        return len(self._images) - 1

    def noise(self, scale):  # NoiseTexture::new (texture.rs:102-104): Perlin::default()
        self._textures.append(N.gs_texture_spec(kind=N.GS_TEX_NOISE, a=-1, b=-1, p=(scale, 0.0, 0.0)))
        return len(self._textures) - 1

    def image_texture(self, image_index):
        self._textures.append(N.gs_texture_spec(kind=N.GS_TEX_IMAGE, a=image_index, b=-1))
        return len(self._textures) - 1

    # ------------------------------------------------------------ materials
    def _mat(self, kind, texture=-1, p=(0.0, 0.0, 0.0, 0.0)):
        m = N.gs_material_spec(kind=kind, texture=texture)
        m.p[:] = [float(x) for x in p]
        self._materials.append(m)
        return len(self._materials) - 1

    def lambertian_texture(self, tex):
        return self._mat(N.GS_MAT_LAMBERTIAN, tex)

    def lambertian(self, rgb):  # Lambertian::from_color
        return self._mat(N.GS_MAT_LAMBERTIAN, self.solid(rgb))

    def metal(self, albedo, fuzz):
        return self._mat(N.GS_MAT_METAL, -1, (albedo[0], albedo[1], albedo[2], fuzz))

    def dielectric(self, refraction_index):
        return self._mat(N.GS_MAT_DIELECTRIC, -1, (refraction_index, 0, 0, 0))

    def diffuse_light(self, rgb):  # DiffuseLight::from_color
        return self._mat(N.GS_MAT_DIFFUSE_LIGHT, self.solid(rgb))

    def isotropic_texture(self, tex):  # Isotropic::new (material.rs:176-178)
        return self._mat(N.GS_MAT_ISOTROPIC, tex)

    def isotropic(self, rgb):  # Isotropic::from_color (material.rs:180-182)
        return self._mat(N.GS_MAT_ISOTROPIC, self.solid(rgb))

    # -------------------------------------------------------------- objects
    def _obj(self, kind, material=-1, first=-1, count=0, p=()):
        o = N.gs_object(kind=kind, material=material, first=first, count=count)
        for k, x in enumerate(p):
            o.p[k] = float(x)
        self._objects.append(o)
        return len(self._objects) - 1

    def sphere(self, center, radius, material):
        return self._obj(N.GS_OBJ_SPHERE, material, p=(*center, radius))

    def moving_sphere(self, c1, c2, radius, material):
        return self._obj(N.GS_OBJ_MOVING_SPHERE, material, p=(*c1, *c2, radius))

    def quad(self, q, u, v, material):
        return self._obj(N.GS_OBJ_QUAD, material, p=(*q, *u, *v))

    def triangle(self, a, b, c, material):
        return self._obj(N.GS_OBJ_TRIANGLE, material, p=(*a, *b, *c))

    def cube(self, a, b, material):  # Quad::cube -> HittableList of 6 quads
        return self._obj(N.GS_OBJ_CUBE, material, p=(*a, *b))

    def _group(self, kind, members):
        first = len(self._children)
        self._children.extend(int(m) for m in members)
        return self._obj(kind, first=first, count=len(members))

    def hittable_list(self, members):
        return self._group(N.GS_OBJ_LIST, members)

    def bvh(self, members):  # BVHNode::from_list of a nested list
        return self._group(N.GS_OBJ_BVH, members)

    def translate(self, obj, offset):
        return self._obj(N.GS_OBJ_TRANSLATE, first=obj, p=tuple(offset))

    def rotate_y(self, obj, angle_degrees):
        return self._obj(N.GS_OBJ_ROTATE_Y, first=obj, p=(angle_degrees,))

    def medium(self, boundary, density, phase_material):  # ConstantMedium::new (volume.rs:17-21)
        return self._obj(N.GS_OBJ_MEDIUM, phase_material, first=boundary, p=(density,))

    def medium_isotropic(self, boundary, density, rgb):  # ConstantMedium::from_isotropic_color (:23-28)
        return self.medium(boundary, density, self.isotropic(rgb))

    def add(self, obj):  # world.add
        self._world.append(int(obj))
        return obj

    # ------------------------------------------------------------ background
    def background_solid(self, rgb):
        b = N.gs_background_spec(kind=N.GS_BG_SOLID)
        b.color[:] = [float(x) for x in rgb]
        self._bg = b

    def background_hdri(self, rgb_f32, rotation):
        a = np.ascontiguousarray(rgb_f32, dtype=np.float32)
        if a.ndim != 3 or a.shape[2] != 3:
            raise ValueError("HDRI must be HxWx3 float32")
        self._keep.append(a)
        b = N.gs_background_spec(kind=N.GS_BG_HDRI, width=a.shape[1], height=a.shape[0], rgb=a.ctypes.data)
        b.rotation[:] = [float(x) for x in rotation]
        self._bg = b

    def build(self):
        return SceneSpec(self._objects, self._children, self._world, self._materials, self._textures,
                         self._images, self._bg, list(self._keep))


def camera_spec(aspect_ratio, image_width, max_depth, v_fov, look_from, look_at, vup, defocus_angle,
                focus_distance):
    """Camera::new arguments (camera.rs:39-51), minus SampleSettings and Background."""
    c = N.gs_camera_spec(aspect_ratio=float(aspect_ratio), image_width=int(image_width), max_depth=int(max_depth),
                         v_fov=float(v_fov), defocus_angle=float(defocus_angle),
                         focus_distance=float(focus_distance))
    c.look_from[:] = [float(x) for x in look_from]
    c.look_at[:] = [float(x) for x in look_at]
    c.vup[:] = [float(x) for x in vup]
    return c


def sample_settings(confidence, tolerance, batch_size, max_samples):
    return N.gs_sample_settings(confidence=float(confidence), tolerance=float(tolerance),
                                batch_size=int(batch_size), max_samples=int(max_samples))


def fixed_spp(spp):
    """Fixed spp through the adaptive sampler: one batch of spp, then n > max breaks."""
    return sample_settings(0.95, 0.0, spp, spp - 1)
