#!/usr/bin/env python3
"""Pack the reference's per-clip CSV quadruple into one binary `.clip` file per motion.

Reference data: `/root/reference/Joints CSV With Hand/<clip>{JointPosRad,JointSpeedRadSec,
JointPosRadRelative,JointVecFromHip}.csv`, read by `low_level_env.py:58-70` with `pandas.read_csv`.
The CSVs are parsed with pandas here too, so every table value is bit-identical to what the reference
env looks up with `DataFrame.iloc[frame][column]`.

`.clip` layout (little endian; see `ilrl_amd/clips.py` for the reader and `include/humanoid_env.h`
`hum_env_set_clip` for the device upload):

    char[8]  magic "HUMCLIP1"
    u32      n_pos, n_vel, n_rel, n_ep        rows of the four tables
    u32      n_jcol (=14), n_ecol (=27)
    u32      name_len; char[name_len] JSON {"clip": ..., "joint_cols": [...], "ep_cols": [...]}
    f64      pos[n_pos][n_jcol], vel[n_vel][n_jcol], rel[n_rel][n_jcol], ep[n_ep][n_ecol]
"""
import argparse
import json
import os
import struct

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
DEFAULT_SRC = "/root/reference/Joints CSV With Hand"
CLIPS = ["motion02_04", "motion08_03", "motion09_03", "motion13_13"]
JOINT_COLS = ["rightHipX", "rightHipY", "rightHipZ", "rightKnee", "leftHipX", "leftHipY", "leftHipZ",
              "leftKnee", "rightShoulderX", "rightShoulderY", "rightElbow", "leftShoulderX", "leftShoulderY",
              "leftElbow"]
EP_PARTS = ["LeftLeg", "LeftFoot", "RightLeg", "RightFoot", "Head", "LeftForeArm", "LeftHand",
            "RightForeArm", "RightHand"]
EP_COLS = ["%s_%sposition" % (p, a) for p in EP_PARTS for a in "XYZ"]


def pack(src, clip, out_dir):
    t = {}
    for key, suffix, cols in (("pos", "JointPosRad", JOINT_COLS), ("vel", "JointSpeedRadSec", JOINT_COLS),
                              ("rel", "JointPosRadRelative", JOINT_COLS), ("ep", "JointVecFromHip", EP_COLS)):
        df = pd.read_csv(os.path.join(src, "%s%s.csv" % (clip, suffix)))
        missing = [c for c in cols if c not in df.columns]
        assert not missing, (clip, suffix, missing)
        t[key] = np.ascontiguousarray(df[cols].to_numpy(dtype=np.float64))
    meta = json.dumps({"clip": clip, "joint_cols": JOINT_COLS, "ep_cols": EP_COLS}).encode()
    path = os.path.join(out_dir, clip + ".clip")
    with open(path, "wb") as f:
        f.write(b"HUMCLIP1")
        f.write(struct.pack("<6I", len(t["pos"]), len(t["vel"]), len(t["rel"]), len(t["ep"]),
                            len(JOINT_COLS), len(EP_COLS)))
        f.write(struct.pack("<I", len(meta)))
        f.write(meta)
        for key in ("pos", "vel", "rel", "ep"):
            f.write(t[key].astype("<f8").tobytes())
    return path, {k: v.shape for k, v in t.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=DEFAULT_SRC)
    ap.add_argument("--out", default=os.path.join(PKG, "data", "clips"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for c in CLIPS:
        path, shapes = pack(a.src, c, a.out)
        print(path, shapes)


if __name__ == "__main__":
    main()
