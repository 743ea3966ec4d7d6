#!/usr/bin/env python3
"""fp32 accuracy lab (CPU): the product's per-lane physics formulation (physics.h, host build lab.cpp) stepped in
float from the same states as the fp64 oracle and the fp32 oracle yardstick (oracle/, test infrastructure), per-lane
ratios kernel / same-lane fp32 envelope over the state blocks the observation reads:
  joint_vel = 0.1 |dqd| (obs 9, 11, ...), joint_pos = 2 |dq| / (hi - lo) (obs 8, 10, ...), body = base z, 0.3 v, quat.
Lanes whose fp64 oracle step moves by > 1e-5 under a 2^-24 perturbation of the input are excluded (ill-conditioned,
as tests/test_gpu_scale.py does).

usage: python3 tools/fp32lab/lab.py [--states gpurun_out/fp32ab/states.npz] [--n 512] [--lib /tmp/liblab.so ...]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "oracle")]
import oracle as O  # noqa: E402

SCALE = None


def blocks(d):
    """per-lane block maxima of a state difference d [n, 47]"""
    jv = 0.1 * np.abs(d[:, 30:47]).max(1)
    jp = (2 * np.abs(d[:, 13:30]) / (O.HI - O.LO)).max(1)
    body = np.maximum.reduce([np.abs(d[:, 2]), 0.3 * np.abs(d[:, 7:10]).max(1), np.abs(d[:, 3:7]).max(1)])
    return {"body": body, "joint_pos": jp, "joint_vel": jv}


def load_lab(path):
    lib = ctypes.CDLL(path)
    dp = ctypes.POINTER(ctypes.c_double)
    for f in ("lab_step_f32", "lab_step_f64"):
        getattr(lib, f).argtypes = [dp, dp]
    return lib


def p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--states", default=os.path.join(REPO, "gpurun_out", "fp32ab", "states.npz"))
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--lib", nargs="+", default=["/tmp/liblab.so"])
    ap.add_argument("--cache", default="/tmp/fp32lab_ref.npz")
    ap.add_argument("--renorm", action="store_true", help="renormalise the base quaternion (float64) first")
    a = ap.parse_args()
    z = np.load(a.states)
    phys, act = z["phys"], z["a"]
    lanes = np.linspace(0, len(phys) - 1, a.n).astype(int)
    tau = np.array([O.motor_torques(act[i]) for i in lanes]).astype(np.float32).astype(np.float64)
    st0 = phys[lanes].astype(np.float64)
    if a.renorm:
        st0[:, 3:7] /= np.linalg.norm(st0[:, 3:7], axis=1, keepdims=True)
        a.cache = a.cache.replace(".npz", "_renorm.npz")
    key = np.array([float(np.sum(st0 * np.arange(1, st0.size + 1).reshape(st0.shape))), float(np.sum(tau))])
    if os.path.exists(a.cache) and np.array_equal(np.load(a.cache)["key"], key):
        c = np.load(a.cache)
        ref, o32, env, sens = c["ref"], c["o32"], c["env"], c["sens"]
    else:
        rng32, rng = np.random.default_rng(7), np.random.default_rng(6)
        ref = np.array([O.phys_step(st0[j], tau[j]) for j in range(len(lanes))])
        o32 = np.array([O.phys_step(st0[j], tau[j], precision="fp32") for j in range(len(lanes))])
        env = {k: np.zeros(len(lanes)) for k in ("body", "joint_pos", "joint_vel")}
        for rz in range(4):
            if rz == 0:
                r = o32
            else:
                r = np.array([O.phys_step(st0[j] * (1 + 2.0 ** -24 * rng32.choice([-1.0, 1.0], 47)), tau[j],
                                          precision="fp32") for j in range(len(lanes))])
            for k, v in blocks(r - ref).items():
                env[k] = np.maximum(env[k], v)
        pert = np.array([O.phys_step(st0[j] * (1 + 2.0 ** -24 * rng.choice([-1.0, 1.0], 47)), tau[j])
                         for j in range(len(lanes))])
        sens = np.abs(pert - ref)[:, 7:47].max(1)
        env = np.stack([env["body"], env["joint_pos"], env["joint_vel"]], 1)
        np.savez(a.cache, key=key, ref=ref, o32=o32, env=env, sens=sens)
    good = sens <= 1e-5 * 10
    print("lanes %d, well-conditioned %d" % (len(lanes), good.sum()))
    envd = {"body": env[:, 0], "joint_pos": env[:, 1], "joint_vel": env[:, 2]}
    rows = {"fp32_oracle": blocks(o32 - ref)}
    for spec in a.lib:
        path, _, mode = spec.partition("@")   # path@mode: lab_set_mode(mode) of an instrumented build
        lib = load_lab(path)
        if mode:
            lib.lab_set_mode(int(mode))
        for prec in ("f32", "f64"):
            out = st0.copy()
            for j in range(len(lanes)):
                getattr(lib, "lab_step_" + prec)(p(out[j]), p(tau[j]))
            rows["%s:%s" % (os.path.basename(spec), prec)] = blocks(out - ref)
    for b in ("body", "joint_pos", "joint_vel"):
        print("== %s   (envelope: max %.2e p50 %.2e)" % (b, envd[b][good].max(), np.median(envd[b][good])))
        for name, bl in rows.items():
            x = bl[b][good]
            r = x / np.maximum(envd[b][good], 1e-9)
            print("  %-24s max %.2e p50 %.2e | ratio p50 %.2f p90 %.2f p99 %.2f max %.2f" % (
                name, x.max(), np.median(x), np.median(r), np.percentile(r, 90), np.percentile(r, 99), r.max()))


if __name__ == "__main__":
    main()
