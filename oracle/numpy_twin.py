"""numpy twin of the CPU oracle — an independent restatement for cross-checking.

TEST INFRASTRUCTURE ONLY (tests/ import it; the product never does).
PARITY STATUS: unpinned against the reference binary.  The
reference's UKF arithmetic lives in ukfom/MTK (absent here).  This twin is
written from the frozen spec in vectorised numpy form — LAPACK
Cholesky, matrix products over all sigma points at once — so that it shares no
code path with oracle/uwvk_oracle.c.  Agreement of the two restatements is the
strongest available guard against a restatement bug.

Sources restated: PoseUKF.cpp:12-84 (process), :107-219 (measurements),
:288-372 (init), :393-465 (noise / predict), :476-611 (update wiring, gates),
:685-699; VelocityUKF.cpp:6-130; PoseState.hpp:29-45.
"""
import numpy as np

EARTHW = 7.292115e-5
A_WGS, F_WGS = 6378137.0, 1.0 / 298.257223563
D2P95 = 5.991
IDX = [0, 1, 5]


# ---------------------------------------------------------------- SO3 / quats
def qmul(a, b):
    a, b = np.asarray(a), np.asarray(b)
    w1, v1 = a[..., :1], a[..., 1:]
    w2, v2 = b[..., :1], b[..., 1:]
    w = w1 * w2 - np.sum(v1 * v2, -1, keepdims=True)
    v = w1 * v2 + w2 * v1 + np.cross(v1, v2)
    return np.concatenate([w, v], -1)


def qconj(q):
    return np.concatenate([q[..., :1], -q[..., 1:]], -1)


def qrot(q, v):
    """Rotate v by unit quaternion q (Eigen _transformVector form)."""
    u = q[..., 1:]
    uv = 2.0 * np.cross(u, v)
    return v + q[..., :1] * uv + np.cross(u, uv)


def qmat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def so3_exp(v):
    v = np.asarray(v, dtype=float)
    th = np.linalg.norm(v, axis=-1, keepdims=True)
    safe = np.where(th > 0, th, 1.0)
    s = np.where(th > 0, np.sin(0.5 * th) / safe, 0.0)
    c = np.where(th > 0, np.cos(0.5 * th), 1.0)
    return np.concatenate([c, s * v], -1)


def so3_log(q):
    q = np.where(q[..., :1] < 0, -q, q)
    nv = np.linalg.norm(q[..., 1:], axis=-1, keepdims=True)
    safe = np.where(nv > 0, nv, 1.0)
    k = np.where(nv > 0, 2.0 * np.arctan2(nv, q[..., :1]) / safe, 0.0)
    return k * q[..., 1:]


# ---------------------------------------------------------------- layout
# SO3 [+] side, process-wide like the C oracle's switch:
# True = body frame q exp(d) (default since r05, MTK's SO3::boxplus), False =
# nav frame exp(d) q.  Set it before constructing a twin.
SO3_RIGHT = True


def so3_plus(q, d, right):
    """q [+] d for an already scaled rotation vector d."""
    return qmul(q, so3_exp(d)) if right else qmul(so3_exp(d), q)


def so3_minus(a, b, right):
    """a [-] b: log(b^-1 a) (right) or log(a b^-1) (left)."""
    return so3_log(qmul(qconj(b), a)) if right else so3_log(qmul(a, qconj(b)))


class Layout:
    def __init__(self, dof, right=None):
        self.dof = dof
        self.right = SO3_RIGHT if right is None else right
        self.full = dof == 53
        self.store = dof + 1
        # tangent -> storage for vect DOFs
        self.vec_d = np.array([d for d in range(dof) if not 3 <= d < 6])
        self.vec_s = np.where(self.vec_d < 3, self.vec_d, self.vec_d + 1)
        o = 20 if not self.full else 47
        self.s = dict(pos=0, quat=3, vel=7, acc=10, bg=13, ba=16, grav=19, wv=o, wvb=o + 2, badcp=o + 4,
                      rho=o + 6)
        if self.full:
            self.s.update(inertia=20, lin=29, quad=38)
        od = 19 if not self.full else 46
        self.d = dict(pos=0, ori=3, vel=6, acc=9, bg=12, ba=15, grav=18, wv=od, wvb=od + 2, badcp=od + 4,
                      rho=od + 6)
        if self.full:
            self.d.update(inertia=19, lin=28, quad=37)

    def boxplus(self, X, D):
        """X [..., store] (+) D [..., dof]: vect + D; SO3 q exp(D) (right) or exp(D) q (left)."""
        Y = np.array(X, dtype=float, copy=True)
        Y[..., self.vec_s] = X[..., self.vec_s] + D[..., self.vec_d]
        Y[..., 3:7] = so3_plus(X[..., 3:7], D[..., 3:6], self.right)
        return Y

    def boxminus(self, X, M):
        D = np.zeros(X.shape[:-1] + (self.dof,))
        D[..., self.vec_d] = X[..., self.vec_s] - M[..., self.vec_s]
        D[..., 3:6] = so3_minus(X[..., 3:7], M[..., 3:7], self.right)
        return D


class VecLayout:
    def __init__(self, n):
        self.dof = n

    def boxplus(self, X, D):
        return X + D

    def boxminus(self, X, M):
        return X - M


# ---------------------------------------------------------------- UKF core
def sigma_points(lay, mu, P):
    L = np.linalg.cholesky(P)
    n = lay.dof
    D = np.zeros((2 * n + 1, n))
    D[1::2] = L.T
    D[2::2] = -L.T
    return lay.boxplus(np.broadcast_to(mu, (2 * n + 1,) + mu.shape), D)


def manifold_mean(lay, X):
    ref = X[0].copy()
    for _ in range(10000):
        d = lay.boxminus(X, ref).mean(axis=0)
        ref = lay.boxplus(ref, d)
        if np.linalg.norm(d) <= 1e-6:
            break
    return ref


def vect_mean(Z):
    ref = Z[0].copy()
    for _ in range(10000):
        d = (Z - ref).mean(axis=0)
        ref = ref + d
        if np.linalg.norm(d) <= 1e-6:
            break
    return ref


def ukf_predict(lay, mu, P, g, Qp):
    X = sigma_points(lay, mu, P)
    X = g(X)
    m = manifold_mean(lay, X)
    D = lay.boxminus(X, m)
    return m, 0.5 * D.T @ D + Qp


def ukf_update(lay, mu, P, z, h, R, zmanifold, gate):
    X = sigma_points(lay, mu, P)
    Z = h(X)
    zm = vect_mean(Z) if zmanifold else Z.mean(axis=0)
    dZ = Z - zm
    dX = lay.boxminus(X, mu)
    S = 0.5 * dZ.T @ dZ + R
    C = 0.5 * dX.T @ dZ
    Si = np.linalg.inv(S)
    K = C @ Si
    nu = z - zm
    d2 = nu @ Si @ nu
    if gate and d2 > D2P95:
        return mu, P, False
    P = P - C @ K.T
    delta = K @ nu
    # apply_delta: re-spread, shift by delta, covariance about mu [+] delta
    X = sigma_points(lay, mu, P)
    mu = lay.boxplus(mu, delta)
    X = lay.boxplus(X, np.broadcast_to(delta, (X.shape[0], delta.shape[0])))
    D = lay.boxminus(X, mu)
    return mu, 0.5 * D.T @ D, True


# ---------------------------------------------------------------- geography
def radii(lat0):
    e2 = F_WGS * (2 - F_WGS)
    den = 1 - e2 * np.sin(lat0) ** 2
    return A_WGS * (1 - e2) / den ** 1.5, A_WGS / np.sqrt(den)


def nav_to_world(loc, x, y):
    rm, rn = radii(loc[0])
    return loc[0] + x / rm, loc[1] - y / (rn * np.cos(loc[0]))


def world_to_nav(loc, lat, lon):
    rm, rn = radii(loc[0])
    return (lat - loc[0]) * rm, -(lon - loc[1]) * rn * np.cos(loc[0])


def wgs84_gravity(lat, alt):
    s2 = np.sin(lat) ** 2
    return 9.7803253359 * (1 + 0.00193185265241 * s2) / np.sqrt(1 - 0.00669437999013 * s2) - 3.086e-6 * alt


# ---------------------------------------------------------------- dynamics
class UWV:
    def __init__(self, M, Dl, Dq, weight=0.0, buoyancy=0.0, cog=(0, 0, 0), cob=(0, 0, 0)):
        self.M, self.Dl, self.Dq = np.array(M, float), np.array(Dl, float), np.array(Dq, float)
        self.W, self.B = weight, buoyancy
        self.cog, self.cob = np.array(cog, float), np.array(cob, float)

    @classmethod
    def from_abi(cls, u):
        return cls(np.array(u.inertia_matrix[:]).reshape(6, 6), np.array(u.damping_matrices[0][:]).reshape(6, 6),
                   np.array(u.damping_matrices[1][:]).reshape(6, 6), u.weight, u.buoyancy,
                   u.distance_body2centerofgravity[:], u.distance_body2centerofbuoyancy[:])

    def forces(self, M, Dl, Dq, nu, q):
        v, w = nu[..., :3], nu[..., 3:]
        a = nu @ M[:3].T
        b = nu @ M[3:].T
        cor = np.concatenate([np.cross(w, a), np.cross(v, a) + np.cross(w, b)], -1)
        damp = nu @ Dl.T + (np.abs(nu) * nu) @ Dq.T
        qc = qconj(q)
        fg = qrot(qc, np.array([0.0, 0.0, -self.W]))
        fb = qrot(qc, np.array([0.0, 0.0, self.B]))
        g = -np.concatenate([fg + fb, np.cross(self.cog, fg) + np.cross(self.cob, fb)], -1)
        return cor, damp, g

    def efforts(self, acc6, nu, q, M=None, Dl=None, Dq=None):
        M = self.M if M is None else M
        Dl = self.Dl if Dl is None else Dl
        Dq = self.Dq if Dq is None else Dq
        cor, damp, g = self.forces(M, Dl, Dq, nu, q)
        return acc6 @ M.T + cor + damp + g

    def rk4(self, s, tau, dt):
        Minv = np.linalg.inv(self.M)

        def f(s):
            q = s[..., 3:7]
            nu = s[..., 7:13]
            pd = qrot(q, s[..., 7:10])
            wq = np.concatenate([np.zeros(nu.shape[:-1] + (1,)), nu[..., 3:]], -1)
            qd = 0.5 * qmul(q, wq)
            cor, damp, g = self.forces(self.M, self.Dl, self.Dq, nu, q)
            nud = (tau - cor - damp - g) @ Minv.T
            return np.concatenate([pd, qd, nud], -1)

        k1 = f(s)
        k2 = f(s + 0.5 * dt * k1)
        k3 = f(s + 0.5 * dt * k2)
        k4 = f(s + dt * k3)
        o = s + dt / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
        o[..., 3:7] /= np.linalg.norm(o[..., 3:7], axis=-1, keepdims=True)
        return o


# ---------------------------------------------------------------- PoseUKF
class PoseTwin:
    """Single PoseUKF instance (numpy)."""

    def __init__(self, dof, x, P, loc, uwv, param):
        self.lay = Layout(dof)
        self.mu, self.P = np.array(x, float), np.array(P, float)
        self.loc = np.array(loc, float)
        self.uwv = uwv
        self.p = param  # dict of PoseUKFParameter fields
        s = self.lay.s
        if self.lay.full:
            self.off_i = self.mu[s["inertia"]:s["inertia"] + 9].copy()
            self.off_l = self.mu[s["lin"]:s["lin"] + 9].copy()
            self.off_q = self.mu[s["quad"]:s["quad"] + 9].copy()
        self.off_rho = self.mu[s["rho"]]
        self.w = np.zeros(3)
        self.Q = np.zeros((dof, dof))
        self.model_blocks = None  # shared DynamicModel's (surge,sway,yaw) blocks, None = base

    @classmethod
    def from_config(cls, dof, pos, pos_cov, rot, rot_cov, cfg, uwv):
        """PoseUKF.cpp:288-372 with imu_in_body = identity."""
        lay = Layout(dof)
        s, d = lay.s, lay.d
        x = np.zeros(lay.store)
        x[0:3], x[3:7] = pos, rot
        x[s["bg"]:s["bg"] + 3] = cfg["gyro_bias_offset"]
        x[s["ba"]:s["ba"] + 3] = cfg["acc_bias_offset"]
        x[s["grav"]] = wgs84_gravity(cfg["lat"], cfg["alt"])
        if lay.full:
            x[s["inertia"]:s["inertia"] + 9] = uwv.M[np.ix_(IDX, IDX)].ravel(order="F")
            x[s["lin"]:s["lin"] + 9] = uwv.Dl[np.ix_(IDX, IDX)].ravel(order="F")
            x[s["quad"]:s["quad"] + 9] = uwv.Dq[np.ix_(IDX, IDX)].ravel(order="F")
        x[s["rho"]] = cfg["rho"]
        P = np.zeros((dof, dof))
        P[0:3, 0:3], P[3:6, 3:6] = pos_cov, rot_cov
        P[6:9, 6:9], P[9:12, 9:12] = np.eye(3), 10 * np.eye(3)
        P[12:15, 12:15] = np.diag(np.square(cfg["gyro_bias_instability"]))
        P[15:18, 15:18] = np.diag(np.square(cfg["acc_bias_instability"]))
        P[18, 18] = 0.05 ** 2
        if lay.full:
            for k in ("inertia", "lin", "quad"):
                P[d[k]:d[k] + 9, d[k]:d[k] + 9] = np.diag(np.square(cfg[k + "_instability"]))
        for k in ("wv", "wvb"):
            P[d[k]:d[k] + 2, d[k]:d[k] + 2] = cfg["wv_limits"] ** 2 * np.eye(2)
        P[d["badcp"]:d["badcp"] + 2, d["badcp"]:d["badcp"] + 2] = cfg["adcp_limits"] ** 2 * np.eye(2)
        P[d["rho"], d["rho"]] = cfg["rho_limits"] ** 2
        param = dict(imu_in_body=np.zeros(3), gyro_bias_offset=np.array(cfg["gyro_bias_offset"]),
                     gyro_bias_tau=cfg["gyro_tau"], acc_bias_offset=np.array(cfg["acc_bias_offset"]),
                     acc_bias_tau=cfg["acc_tau"], inertia_tau=cfg["inertia_tau"], lin_damping_tau=cfg["lin_tau"],
                     quad_damping_tau=cfg["quad_tau"], water_velocity_tau=cfg["wv_tau"],
                     water_velocity_scale=cfg["wv_scale"], adcp_bias_tau=cfg["adcp_tau"],
                     atmospheric_pressure=cfg["patm"], water_density_tau=cfg["rho_tau"])
        f = cls(dof, x, P, (cfg["lat"], cfg["lon"]), uwv, param)
        return f

    def set_noise_from_config(self, cfg, dt):
        """PoseUKF.cpp:393-439 (imu_in_body = identity)."""
        lay, d = self.lay, self.lay.d
        Q = np.zeros((lay.dof, lay.dof))
        j = np.asarray(cfg["max_jerk"], float)
        Q[0:3, 0:3] = np.diag(1.5 * dt ** 4 * (j / 24.0) ** 2)
        Q[6:9, 6:9] = np.diag(1.5 * dt ** 2 * (j / 8.0) ** 2)
        Q[9:12, 9:12] = np.diag((j / 4.0) ** 2)
        Q[3:6, 3:6] = np.diag(np.square(cfg["gyro_randomwalk"]))
        Q[12:15, 12:15] = np.diag(2.0 / (cfg["gyro_tau"] * dt) * np.square(cfg["gyro_bias_instability"]))
        Q[15:18, 15:18] = np.diag(2.0 / (cfg["acc_tau"] * dt) * np.square(cfg["acc_bias_instability"]))
        Q[18, 18] = 1e-12
        if lay.full:
            for k, tk in (("inertia", "inertia_tau"), ("lin", "lin_tau"), ("quad", "quad_tau")):
                Q[d[k]:d[k] + 9, d[k]:d[k] + 9] = np.diag(2.0 / (cfg[tk] * dt) * np.square(cfg[k + "_instability"]))
        for k in ("wv", "wvb"):
            Q[d[k]:d[k] + 2, d[k]:d[k] + 2] = 2.0 / (cfg["wv_tau"] * dt) * cfg["wv_limits"] ** 2 * np.eye(2)
        Q[d["badcp"]:d["badcp"] + 2, d["badcp"]:d["badcp"] + 2] = (2.0 / (cfg["adcp_tau"] * dt) *
                                                                   cfg["adcp_limits"] ** 2 * np.eye(2))
        Q[d["rho"], d["rho"]] = 2.0 / (cfg["rho_tau"] * dt) * cfg["rho_limits"] ** 2
        self.Q = Q

    # -- process model, PoseUKF.cpp:12-84 (vectorised over sigma points)
    def _g(self, X, dt):
        s, p = self.lay.s, self.p
        Y = X.copy()
        Y[:, 0:3] = X[:, 0:3] + dt * X[:, 7:10]
        lat, _ = nav_to_world(self.loc, X[:, 0], X[:, 1])
        er = EARTHW * np.stack([np.cos(lat), np.zeros_like(lat), np.sin(lat)], -1)
        wn = qrot(X[:, 3:7], self.w - X[:, s["bg"]:s["bg"] + 3]) - er
        Y[:, 3:7] = so3_plus(X[:, 3:7], wn * dt, self.lay.right)  # orientation.boxplus, :32
        Y[:, 7:10] = X[:, 7:10] + dt * X[:, 10:13]

        def decay(sl, tau, off):
            Y[:, sl] = X[:, sl] + dt * ((-1.0 / tau) * (X[:, sl] - off))

        decay(slice(s["bg"], s["bg"] + 3), p["gyro_bias_tau"], p["gyro_bias_offset"])
        decay(slice(s["ba"], s["ba"] + 3), p["acc_bias_tau"], p["acc_bias_offset"])
        if self.lay.full:
            decay(slice(s["inertia"], s["inertia"] + 9), p["inertia_tau"], self.off_i)
            decay(slice(s["lin"], s["lin"] + 9), p["lin_damping_tau"], self.off_l)
            decay(slice(s["quad"], s["quad"] + 9), p["quad_damping_tau"], self.off_q)
        decay(slice(s["wv"], s["wv"] + 4), p["water_velocity_tau"], 0.0)
        decay(slice(s["badcp"], s["badcp"] + 2), p["adcp_bias_tau"], 0.0)
        decay(slice(s["rho"], s["rho"] + 1), p["water_density_tau"], self.off_rho)
        return Y

    def predict(self, dt):
        """predictionStepImpl, PoseUKF.cpp:446-465."""
        d = self.lay.d
        Qp = self.Q.copy()
        R = qmat(self.mu[3:7])
        Qp[3:6, 3:6] = R @ self.Q[3:6, 3:6] @ R.T
        vs = self.mu[7:10] * np.array([1, 1, 10.0])
        add = self.p["water_velocity_scale"] * (vs @ vs) * dt
        for k in ("wv", "wvb"):
            Qp[d[k]:d[k] + 2, d[k]:d[k] + 2] += add * np.eye(2)
        self.mu, self.P = ukf_predict(self.lay, self.mu, self.P, lambda X: self._g(X, dt), dt ** 2 * Qp)

    def _upd(self, z, h, R, zman, gate=False):
        self.mu, self.P, acc = ukf_update(self.lay, self.mu, self.P, np.asarray(z, float), h,
                                          np.asarray(R, float), zman, gate)
        return acc

    def rotation_rate_body(self):
        """getRotationRate, PoseUKF.cpp:693-699."""
        lat, _ = nav_to_world(self.loc, self.mu[0], self.mu[1])
        er = EARTHW * np.array([np.cos(lat), 0.0, np.sin(lat)])
        return self.w - self.mu[self.lay.s["bg"]:self.lay.s["bg"] + 3] - qrot(qconj(self.mu[3:7]), er)

    def update(self, kind, z, R, extra=None, only_vel=False):
        s = self.lay.s
        if kind == "acceleration":
            return self._upd(z, lambda X: qrot(qconj(X[:, 3:7]), X[:, 10:13] + np.outer(X[:, s["grav"]], [0, 0, 1]))
                             + X[:, s["ba"]:s["ba"] + 3], R, True)
        if kind == "velocity":
            return self._upd(z, lambda X: qrot(qconj(X[:, 3:7]), X[:, 7:10]), R, True)
        if kind == "pressure":
            sp = np.zeros(3) if extra is None else np.asarray(extra, float)
            return self._upd(z, lambda X: (self.p["atmospheric_pressure"] - (X[:, 2] + qrot(X[:, 3:7], sp)[:, 2]) *
                                           X[:, s["grav"]] * X[:, s["rho"]])[:, None], R, False)
        if kind == "water_velocity":
            cw = float(extra)

            def h(X):
                qi = qconj(X[:, 3:7])
                v = X[:, 7:10]
                wvb = np.concatenate([X[:, s["wvb"]:s["wvb"] + 2], np.zeros((len(X), 1))], 1)
                wv = np.concatenate([X[:, s["wv"]:s["wv"] + 2], np.zeros((len(X), 1))], 1)
                return (cw * qrot(qi, v - wvb) + (1 - cw) * qrot(qi, v - wv))[:, :2] + X[:, s["badcp"]:s["badcp"] + 2]
            return self._upd(z, h, R, True, gate=True)
        if kind == "xy":
            return self._upd(z, lambda X: X[:, 0:2], R, False)
        if kind == "z":
            return self._upd(z, lambda X: X[:, 2:3], R, False)
        if kind == "geographic":
            gps = np.zeros(3) if extra is None else np.asarray(extra, float)
            x, y = world_to_nav(self.loc, z[0], z[1])
            zz = np.array([x, y]) - qrot(self.mu[3:7], gps)[:2]
            return self._upd(zz, lambda X: X[:, 0:2], R, False, gate=True)
        if kind == "delayed_xy":
            zz = np.asarray(z, float) + (self.mu[0:2] - np.asarray(extra, float))
            return self._upd(zz, lambda X: X[:, 0:2], R, False)
        if kind == "efforts":
            return self._efforts(z, R, only_vel)
        raise KeyError(kind)

    def _blocks(self, blk):
        M, Dl, Dq = self.uwv.M.copy(), self.uwv.Dl.copy(), self.uwv.Dq.copy()
        if blk is not None:
            for mat, k in ((M, 0), (Dl, 1), (Dq, 2)):
                mat[np.ix_(IDX, IDX)] = blk[9 * k:9 * k + 9].reshape(3, 3, order="F")
        return M, Dl, Dq

    def _efforts(self, z, R, only_vel):
        """PoseUKF.cpp:153-219, 581-602."""
        s = self.lay.s
        wb = self.rotation_rate_body()
        imu = self.p["imu_in_body"]
        if only_vel:
            q = self.mu[3:7]
            w3 = np.array([self.mu[s["wv"]], self.mu[s["wv"] + 1], 0.0])
            ab = qrot(qconj(q), self.mu[10:13]) - np.cross(wb, np.cross(wb, imu))
            M, Dl, Dq = self._blocks(self.model_blocks)

            def h(X):
                vb = qrot(qconj(q), X[:, 7:10]) - np.cross(wb, imu) - qrot(qconj(q), w3)
                nu = np.concatenate([vb, np.broadcast_to(wb, vb.shape)], 1)
                acc6 = np.concatenate([np.broadcast_to(ab, vb.shape), np.zeros_like(vb)], 1)
                return np.stack([self.uwv.efforts(acc6[i], nu[i], q, M, Dl, Dq) for i in range(len(X))])
            return self._upd(z, h, R, False)

        def h(X):
            out = []
            for x in X:
                blk = None
                if self.lay.full:
                    blk = np.concatenate([x[s["inertia"]:s["inertia"] + 9], x[s["lin"]:s["lin"] + 9],
                                          x[s["quad"]:s["quad"] + 9]])
                M, Dl, Dq = self._blocks(blk)
                qi = qconj(x[3:7])
                wv = np.array([x[s["wv"]], x[s["wv"] + 1], 0.0])
                vb = qrot(qi, x[7:10]) - np.cross(wb, imu) - qrot(qi, wv)
                ab = qrot(qi, x[10:13]) - np.cross(wb, np.cross(wb, imu))
                out.append(self.uwv.efforts(np.concatenate([ab, np.zeros(3)]), np.concatenate([vb, wb]), x[3:7],
                                            M, Dl, Dq))
                if self.lay.full:
                    self.model_blocks = blk  # the shared model keeps the last point's blocks (:173)
            return np.stack(out)
        return self._upd(z, h, R, False)


# ---------------------------------------------------------------- VelocityUKF
class VelTwin:
    def __init__(self, x, P, uwv):
        self.lay = VecLayout(4)
        self.mu, self.P = np.array(x, float), np.array(P, float)
        self.Q = np.diag([1e-4, 1e-4, 1e-4, 0.0])
        self.uwv = uwv
        self.gyro = np.zeros(3)
        self.tau = np.zeros(6)
        self.model = np.concatenate([np.zeros(3), [1.0, 0, 0, 0], self.mu[:3], self.gyro])

    def set_gyro(self, w):
        self.gyro = np.asarray(w, float)
        self.model[10:13] = self.gyro

    def predict(self, dt):
        q = self.model[3:7]

        def g(X):
            s = np.concatenate([np.zeros((len(X), 3)), np.broadcast_to(q, (len(X), 4)), X[:, :3],
                                np.broadcast_to(self.gyro, (len(X), 3))], 1)
            n = self.uwv.rk4(s, self.tau, dt)
            v = X[:, :3] + (n[:, 7:10] - X[:, :3])
            z = X[:, 3] + dt * qrot(q, v)[:, 2]
            return np.concatenate([v, z[:, None]], 1)
        self.mu, self.P = ukf_predict(self.lay, self.mu, self.P, g, dt * self.Q)
        self.model = self.uwv.rk4(self.model, self.tau, dt)

    def update_dvl(self, z, R):
        self.mu, self.P, _ = ukf_update(self.lay, self.mu, self.P, np.asarray(z, float), lambda X: X[:, :3],
                                        np.asarray(R, float), True, False)

    def update_pressure(self, z, R):
        self.mu, self.P, _ = ukf_update(self.lay, self.mu, self.P, np.atleast_1d(np.asarray(z, float)),
                                        lambda X: X[:, 3:4], np.atleast_2d(R), True, False)


def cfg_dict(c):
    """Flatten an abi.PoseConfig into the dict PoseTwin.from_config expects."""
    m = c.model_noise_parameters
    return dict(gyro_bias_offset=list(c.rotation_rate.bias_offset), acc_bias_offset=list(c.acceleration.bias_offset),
                gyro_bias_instability=list(c.rotation_rate.bias_instability),
                acc_bias_instability=list(c.acceleration.bias_instability),
                gyro_randomwalk=list(c.rotation_rate.randomwalk), gyro_tau=c.rotation_rate.bias_tau,
                acc_tau=c.acceleration.bias_tau, lat=c.location.latitude, lon=c.location.longitude,
                alt=c.location.altitude, rho=c.hydrostatics.water_density,
                rho_limits=c.hydrostatics.water_density_limits, rho_tau=c.hydrostatics.water_density_tau,
                patm=c.hydrostatics.atmospheric_pressure, inertia_instability=list(m.inertia_instability),
                lin_instability=list(m.lin_damping_instability), quad_instability=list(m.quad_damping_instability),
                inertia_tau=m.inertia_tau, lin_tau=m.lin_damping_tau, quad_tau=m.quad_damping_tau,
                wv_limits=c.water_velocity.limits, wv_tau=c.water_velocity.tau, wv_scale=c.water_velocity.scale,
                adcp_limits=c.water_velocity.adcp_bias_limits, adcp_tau=c.water_velocity.adcp_bias_tau,
                max_jerk=list(c.max_jerk))
