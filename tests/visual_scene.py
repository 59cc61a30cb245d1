"""Synthetic marker scenes for the visual-landmark updates (test helper).

A square marker (4 corners, half size 0.2 m) 3 m ahead of the camera; the
camera looks along the body x axis (camera z forward, x right, y down).
Image coordinates are the undistorted pinhole projection of the true corners
plus seeded pixel noise."""
import numpy as np

CAMERA = np.array([600.0, 620.0, 320.0, 240.0])  # fx, fy, cx, cy
CORNERS = 0.2 * np.array([[1.0, 1.0, 0.0], [-1.0, 1.0, 0.0], [-1.0, -1.0, 0.0], [1.0, -1.0, 0.0]])


def qmul(a, b):
    aw, ax, ay, az = a[..., 0], a[..., 1], a[..., 2], a[..., 3]
    bw, bx, by, bz = b[..., 0], b[..., 1], b[..., 2], b[..., 3]
    return np.stack([aw * bw - ax * bx - ay * by - az * bz, aw * bx + ax * bw + ay * bz - az * by,
                     aw * by + ay * bw + az * bx - ax * bz, aw * bz + az * bw + ax * by - ay * bx], -1)


def qrot(q, v):
    qv = np.concatenate([np.zeros(v.shape[:-1] + (1,)), v], -1)
    qc = q * np.array([1.0, -1.0, -1.0, -1.0])
    return qmul(qmul(q, qv), qc)[..., 1:]


def qexp(rv):
    th = np.linalg.norm(rv, axis=-1, keepdims=True)
    s = np.where(th > 0, np.sin(th / 2) / np.where(th > 0, th, 1), 0.5)
    return np.concatenate([np.cos(th / 2), s * rv], -1)


def mat_to_quat(R):
    w = np.sqrt(max(0.0, 1 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    x = np.copysign(np.sqrt(max(0.0, 1 + R[0, 0] - R[1, 1] - R[2, 2])) / 2, R[2, 1] - R[1, 2])
    y = np.copysign(np.sqrt(max(0.0, 1 - R[0, 0] + R[1, 1] - R[2, 2])) / 2, R[0, 2] - R[2, 0])
    z = np.copysign(np.sqrt(max(0.0, 1 - R[0, 0] - R[1, 1] + R[2, 2])) / 2, R[1, 0] - R[0, 1])
    return np.array([w, x, y, z])


# camera in body/IMU: 10 cm ahead, z_cam = x_body, x_cam = -y_body, y_cam = -z_body
CAM_IN_BODY = np.concatenate([[0.1, 0.0, 0.05], mat_to_quat(np.array([[0.0, 0.0, 1.0], [-1.0, 0.0, 0.0],
                                                                      [0.0, -1.0, 0.0]]))])


def project(body_t, body_q, marker, cam_in_body=CAM_IN_BODY, corners=CORNERS, camera=CAMERA):
    """pixel coordinates [batch, 4, 2] of the corners for true body poses [batch, 3/4]."""
    fn = qrot(marker[..., None, 3:], corners[None]) + marker[..., None, :3]
    t = qrot(body_q[:, None] * np.array([1.0, -1.0, -1.0, -1.0]), fn - body_t[:, None])
    w = t - cam_in_body[:3]
    fc = qrot(np.broadcast_to(cam_in_body[3:] * np.array([1.0, -1.0, -1.0, -1.0]), w.shape[:-1] + (4,)), w)
    u = camera[0] * fc[..., 0] / fc[..., 2] + camera[2]
    v = camera[1] * fc[..., 1] / fc[..., 2] + camera[3]
    return np.stack([u, v], -1), fc[..., 2]


def marker_ahead(body_t, body_q, dist=3.0):
    """marker pose [batch, 7] dist metres ahead of each body pose, facing it."""
    ahead = body_t + qrot(body_q, np.broadcast_to([dist, 0.0, 0.0], body_t.shape))
    return np.concatenate([ahead, body_q], -1)


def pixel_noise(batch, seed, sigma=0.5):
    return sigma * np.random.default_rng(seed).standard_normal((batch, 4, 2))
