"""Shared parity cases: cameras A/B/C, uniforms variants, frame sizes."""
import numpy as np

import black_hole_ray_marching_amd as bh

CAMERAS = {
    "A": None,                                   # Scene::new default, src/scene.rs:68-76
    "B": ((0.0, 3.0, -20.0), (0.0, 0.0, 0.0)),
    "C": ((0.0, 6.0, -12.0), (0.0, 0.0, 0.0)),
    "D": ((7.0, 1.5, -9.0), (0.0, 0.0, 0.0)),    # off-axis, close: many disc/photon-sphere rays
    "E": ((0.0, 0.0, -20.0), (2.6, 0.0, 0.0), 0.1),  # zoom on the shadow edge: capped "Zeno" rays
    # the camera at the unit sphere (the blackout test's two clauses, :272-283; the kernel's
    # camera-outside step applies for |pos|^2 > 1.01 only, bh_march.hpp SF_CAM_OUT):
    "F": ((0.0, 0.0, -0.5), (0.0, 0.0, -5.0)),   # inside, looking out: escapes, caps and blackouts
    "F2": ((0.2, 0.1, -0.5), (3.0, 1.0, 0.0)),   # inside, sideways: also disc hits
    "G": ((0.0, 0.6, -0.8018), (4.0, 0.6, -0.8)),  # |pos|^2 = 1.0029: outside, general step
    "H": ((0.0, 0.0, -1.02), (3.0, 0.0, -1.0)),  # |pos|^2 = 1.0404: camera-outside step, rays plunge in
}


def camera_uniform(name: str, width: int, height: int) -> bh.CameraUniform:
    spec = CAMERAS[name]
    cam = bh.Camera.default(width, height) if spec is None else bh.Camera.look_at(spec[0], spec[1], width, height)
    if spec is not None and len(spec) > 2:
        cam.fovy = spec[2]
    cu = bh.CameraUniform()
    cu.update(cam)
    return cu


def uniforms(**kw) -> bh.Uniforms:
    u = bh.Uniforms.default()
    for k, v in kw.items():
        setattr(u, k, v)
    return u
