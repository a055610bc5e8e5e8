"""Measurement script (not a test; pytest does not collect it): PCG iteration counts on the reduced camera system of
config 2 / 3 (dense numpy, S and b from the C oracle at LM steps 1-9) for block-Jacobi, the additive two-level
preconditioner of the build (AD), AD with x0 = Q b, A-DEF2 and BNN (Tang, Nabben, Vuik & Erlangga 2009), exact E,
stop rule ||r|| <= 1e-5 ||b||.  Output: profiles/r5_v4/deflation_probe.log.

    python tests/experiments/deflation_probe.py 3
"""
import sys, time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
import numpy as np
from oracle.oracle import OracleBA
from instantsfm_amd.synth import make_config

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
prob = make_config(cfg)
ora = OracleBA(prob.model, prob.uv, prob.cam_idx, prob.pt_idx, prob.pp, prob.n_cams, prob.n_points)
cams = prob.cams_init.copy(); pts = prob.points_init.copy()
C, D = prob.n_cams, ora.D
lab, nc = ora.clusters()
print("C", C, "D", D, "clusters", nc, flush=True)

def quat_R(q):
    x, y, z, w = q
    return np.array([[1-2*(y*y+z*z), 2*(x*y-z*w), 2*(x*z+y*w)],
                     [2*(x*y+z*w), 1-2*(x*x+z*z), 2*(y*z-x*w)],
                     [2*(x*z-y*w), 2*(y*z+x*w), 1-2*(x*x+y*y)]])

def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])

def basis(cams):
    MC = D + 1
    Z = np.zeros((C * D, nc * MC))
    for i in range(C):
        t = cams[i, :3]; R = quat_R(cams[i, 3:7])
        G = np.zeros((D, MC))
        G[0:3, 0:3] = -R
        G[0:3, 3:6] = -skew(t) @ R
        G[0:3, 6] = t
        G[3:6, 3:6] = -R
        for k in range(D - 6):
            G[6 + k, 7 + k] = 1.0
        c = lab[i]
        Z[i*D:(i+1)*D, c*MC:(c+1)*MC] = G
    return Z

def dense_S(f):
    Sb, b = ora.build_reduced(f)
    rp, col = ora.pattern()
    S = np.zeros((C*D, C*D))
    for i in range(C):
        for e in range(rp[i], rp[i+1]):
            j = col[e]
            S[i*D:(i+1)*D, j*D:(j+1)*D] = Sb[e]
            if j != i:
                S[j*D:(j+1)*D, i*D:(i+1)*D] = Sb[e].T
    return S, b.reshape(-1)

def pcg(S, b, Minv, x0=None, tol=1e-5, maxit=500):
    x = np.zeros_like(b) if x0 is None else x0.copy()
    r = b - S @ x
    z = Minv(r); p = z.copy(); rz = r @ z
    # the build's stop rule: ||L^-1 r||^2 <= tol^2 ||L^-1 b||^2 with block-Jacobi scaling -- approximate with ||r||/||b||
    nb = np.linalg.norm(b)
    for it in range(maxit):
        if np.linalg.norm(r) <= tol * nb:
            return it, x
        q = S @ p
        a = rz / (p @ q)
        x += a * p; r -= a * q
        z = Minv(r); rz2 = r @ z
        p = z + (rz2 / rz) * p; rz = rz2
    return maxit, x

STEPS = (1, 5, 8) if cfg == 3 else (1, 4, 7, 9)
for step in range(10):
    if step in STEPS:
        ora.linearize(cams, pts)
        for f in (1.0 + 1e-2, 1.0 + 1e-4):
            S, b = dense_S(f)
            Z = basis(cams)
            blocks = [np.linalg.inv(S[i*D:(i+1)*D, i*D:(i+1)*D]) for i in range(C)]
            def Mbj(r):
                out = np.empty_like(r)
                for i in range(C):
                    out[i*D:(i+1)*D] = blocks[i] @ r[i*D:(i+1)*D]
                return out
            E = Z.T @ S @ Z
            d = np.sqrt(np.diag(E)); d[d == 0] = 1
            Ei = np.linalg.inv(E)
            Q = lambda r: Z @ (Ei @ (Z.T @ r))
            AD = lambda r: Mbj(r) + Q(r)
            def ADEF2(r):
                y = Mbj(r)
                return y - Q(S @ y) + Q(r)
            def BNN(r):
                pr = r - S @ Q(r)
                y = Mbj(pr)
                return y - Q(S @ y) + Q(r)
            x0 = Q(b)
            res = {}
            res["BJ"] = pcg(S, b, Mbj)[0]
            res["AD"] = pcg(S, b, AD)[0]
            res["AD x0=Qb"] = pcg(S, b, AD, x0)[0]
            res["ADEF2 x0=Qb"] = pcg(S, b, ADEF2, x0)[0]
            res["ADEF2 x0=0"] = pcg(S, b, ADEF2)[0]
            res["BNN"] = pcg(S, b, BNN)[0]
            print(f"step {step} f-1={f-1:.0e}: " + ", ".join(f"{k} {v}" for k, v in res.items()), flush=True)
    ora.step(cams, pts)
