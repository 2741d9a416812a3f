"""The scene of the reference's example program (src/main.rs:17-78) on one eray context.

main.rs loads a mesh, builds the example material graph (wave -> rgb, flat_color -> mixer;
main.rs:80-144), sets its inputs (width = height = 1024, x_fac = y_fac = 1, red = 1,
green = 0, blue = 0, factor = 0.5; main.rs:22-41), runs Material::update, and renders with
Engine::new((W, H), 0, 0), a camera at (0, 0, 5) and two lights: ambient (0, 2, 0) with
brightness 0.2 and point (1, 1, 2) with brightness 1 (main.rs:44-65).
"""
from __future__ import annotations

import numpy as np

from . import capi

MAIN_RS_INPUTS = dict(x_fac=1.0, y_fac=1.0, r=1.0, g=0.0, b=0.0, factor=0.5)


def fov_for(width: int, height: int) -> tuple[float, float]:
    """Fov(60, 60) for square frames, Fov(16, 9) for 16:9 (Camera::size must give
    exactly the engine's height)."""
    if width == height:
        return (60.0, 60.0)
    if width * 9 == height * 16:
        return (16.0, 9.0)
    return (float(width), float(height))


class MainScene:
    """Uploads the mesh, evaluates the material on the GPU and configures camera + lights.

    material="textures": Material::update's textures (eray_material_example), sampled per hit
    as the reference does.  material="example": the same graph evaluated at the hit texel
    (eray_scene_set_object_example_material) — bit-identical, no textures."""

    def __init__(self, ctx: capi.Context, positions, normals, uvs, width: int, height: int,
                 texture: int = 1024, fov=None, material: str = "textures"):
        if material not in ("textures", "example"):
            raise ValueError(f"material {material!r}")
        self.ctx = ctx
        self.width, self.height = width, height
        self.texture = texture
        self.color = ctx.empty((texture, texture, 3), np.float32)
        self.diffuse = ctx.empty((texture, texture), np.float32)
        self.evaluate_material()
        ctx.scene_reset()
        cam = capi.make_camera((0.0, 0.0, 5.0), fov or fov_for(width, height), width, 1.0)
        w, h = capi.camera_size(cam)
        if (w, h) != (width, height):
            raise ValueError(f"Camera::size() = {(w, h)} does not match the engine's {(width, height)}")
        ctx.set_camera(cam)
        ctx.add_light(capi.make_light((0.0, 2.0, 0.0), "ambient", (1.0, 1.0, 1.0), 0.2))
        ctx.add_light(capi.make_light((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0))
        idx = ctx.add_object(positions, normals, uvs, color=self.color.image(), diffuse=self.diffuse.image())
        if material == "example":
            i = MAIN_RS_INPUTS
            ctx.set_object_example_material(idx, texture, texture, i["x_fac"], i["y_fac"], i["r"], i["g"], i["b"],
                                            i["factor"])

    def evaluate_material(self) -> None:
        """Material::update of main.rs's graph (one fused pass)."""
        i = MAIN_RS_INPUTS
        self.ctx.material_example(self.texture, self.texture, i["x_fac"], i["y_fac"], i["r"], i["g"],
                                  i["b"], i["factor"], self.color.ptr, self.diffuse.ptr)

    def render(self, out_rgb=None, out_ppm=None, out_face=None, row0=0, rows=None, flags=0) -> None:
        self.ctx.render(self.width, self.height, row0=row0, rows=rows, out_rgb=out_rgb,
                        out_ppm=out_ppm, out_face=out_face, flags=flags)

    def close(self) -> None:
        self.color.free()
        self.diffuse.free()
