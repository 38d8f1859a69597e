"""Camera matrices in the reference's conventions (host-side plumbing for tests and benches).

Restates utils/graphics_utils.py:38-77 (getWorld2View2, getProjectionMatrix, fov2focal,
focal2fov) and the matrix construction of scene/cameras.py:48-57 (row-vector convention:
world_view_transform = W2C^T, full_proj_transform = world_view @ P^T, camera_center =
inverse(world_view)[3, :3]).  Pinned by tests/golden/cameras.npz, generated from the
reference's own functions.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch


def fov2focal(fov: float, pixels: int) -> float:
    return pixels / (2 * math.tan(fov / 2))


def focal2fov(focal: float, pixels: int) -> float:
    return 2 * math.atan(pixels / (2 * focal))


def get_world2view2(R: np.ndarray, t: np.ndarray, translate=np.array([0.0, 0.0, 0.0]), scale: float = 1.0):
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    cam_center = (C2W[:3, 3] + translate) * scale
    C2W[:3, 3] = cam_center
    Rt = np.linalg.inv(C2W)
    return np.float32(Rt)


def get_projection_matrix(znear: float, zfar: float, fovX: float, fovY: float) -> torch.Tensor:
    tanHalfFovY = math.tan(fovY / 2)
    tanHalfFovX = math.tan(fovX / 2)
    top = tanHalfFovY * znear
    bottom = -top
    right = tanHalfFovX * znear
    left = -right
    P = torch.zeros(4, 4)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


@dataclass
class Camera:
    """The fields of scene/cameras.py:Camera that render() reads (gaussian_renderer/__init__.py:33-48)."""
    image_width: int
    image_height: int
    FoVx: float
    FoVy: float
    world_view_transform: torch.Tensor
    projection_matrix: torch.Tensor
    full_proj_transform: torch.Tensor
    camera_center: torch.Tensor
    znear: float = 0.01
    zfar: float = 100.0

    def to(self, device):
        return Camera(self.image_width, self.image_height, self.FoVx, self.FoVy,
                      self.world_view_transform.to(device), self.projection_matrix.to(device),
                      self.full_proj_transform.to(device), self.camera_center.to(device), self.znear, self.zfar)


def make_camera(R: np.ndarray, T: np.ndarray, FoVx: float, FoVy: float, width: int, height: int,
                device="cpu") -> Camera:
    """scene/cameras.py:48-57 with trans = 0, scale = 1."""
    znear, zfar = 0.01, 100.0
    wv = torch.tensor(get_world2view2(R, T)).transpose(0, 1)
    proj = get_projection_matrix(znear=znear, zfar=zfar, fovX=FoVx, fovY=FoVy).transpose(0, 1)
    full = wv.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
    center = wv.inverse()[3, :3]
    cam = Camera(width, height, FoVx, FoVy, wv, proj, full, center, znear, zfar)
    return cam.to(device)


def look_at_origin(position: np.ndarray):
    """COLMAP-style (R, T) for a camera at `position` looking at the origin, +y down in camera space.

    R's columns are the camera axes in world space (R = C2W rotation, the convention of
    scene/dataset_readers.py:82-83 where R = qvec2rotmat(q).T), T = -R^T c.
    """
    c = np.asarray(position, dtype=np.float64)
    z = -c / np.linalg.norm(c)
    y_world = np.array([0.0, 1.0, 0.0])
    x = np.cross(y_world, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z], axis=1)
    T = -R.T @ c
    return R, T
