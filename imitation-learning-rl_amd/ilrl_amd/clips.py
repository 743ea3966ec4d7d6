"""Reader for the packed `.clip` motion files (format: `tools/pack_clips.py`).

A clip holds the four reference tables the env indexes by frame (`low_level_env.py:59-70`):
joint targets (rad), joint target velocities (rad/s), normalised targets, and end points from hip.
"""
import json
import os
import struct
from dataclasses import dataclass

import numpy as np

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "clips")
# the reference's CSV quadruples ("Joints CSV With Hand/", read by low_level_env.py:58-70), shipped as data
CSV_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "csv")
CLIP_NAMES = ["motion02_04", "motion08_03", "motion09_03", "motion13_13"]

# joint_map of LowLevelHumanoidEnv (low_level_env.py:86-101): env joint -> CSV column, dict order.
JOINT_MAP = [
    ("right_knee", "rightKnee"), ("right_hip_x", "rightHipX"), ("right_hip_y", "rightHipY"),
    ("right_hip_z", "rightHipZ"), ("left_knee", "leftKnee"), ("left_hip_x", "leftHipX"),
    ("left_hip_y", "leftHipY"), ("left_hip_z", "leftHipZ"), ("right_shoulder_x", "rightShoulderX"),
    ("right_shoulder_y", "rightShoulderY"), ("right_elbow", "rightElbow"), ("left_shoulder_x", "leftShoulderX"),
    ("left_shoulder_y", "leftShoulderY"), ("left_elbow", "leftElbow"),
]


@dataclass
class Clip:
    name: str
    pos: np.ndarray      # [n_pos, 14] f64, columns = joint_cols
    vel: np.ndarray      # [n_vel, 14]
    rel: np.ndarray      # [n_rel, 14]
    ep: np.ndarray       # [n_ep, 27]
    joint_cols: list
    ep_cols: list

    @property
    def max_frame(self):
        """`len(joints_df) - 1` (low_level_env.py:80-82)."""
        return self.pos.shape[0] - 1

    def jcol(self, name):
        return self.joint_cols.index(name)

    def ecol(self, name):
        return self.ep_cols.index(name)


def load_clip(name_or_path):
    path = name_or_path
    if not os.path.exists(path):
        path = os.path.join(DATA_DIR, name_or_path + ".clip")
    with open(path, "rb") as f:
        buf = f.read()
    if buf[:8] != b"HUMCLIP1":
        raise ValueError("%s: not a HUMCLIP1 file" % path)
    n_pos, n_vel, n_rel, n_ep, n_jcol, n_ecol = struct.unpack_from("<6I", buf, 8)
    (mlen,) = struct.unpack_from("<I", buf, 32)
    meta = json.loads(buf[36:36 + mlen].decode())
    off = 36 + mlen
    arrs = []
    for rows, cols in ((n_pos, n_jcol), (n_vel, n_jcol), (n_rel, n_jcol), (n_ep, n_ecol)):
        a = np.frombuffer(buf, dtype="<f8", count=rows * cols, offset=off).reshape(rows, cols).copy()
        off += rows * cols * 8
        arrs.append(a)
    return Clip(meta["clip"], *arrs, meta["joint_cols"], meta["ep_cols"])


JOINT_COLS = ["rightHipX", "rightHipY", "rightHipZ", "rightKnee", "leftHipX", "leftHipY", "leftHipZ", "leftKnee",
              "rightShoulderX", "rightShoulderY", "rightElbow", "leftShoulderX", "leftShoulderY", "leftElbow"]
EP_COLS = ["%s_%sposition" % (p, a) for p in ("LeftLeg", "LeftFoot", "RightLeg", "RightFoot", "Head", "LeftForeArm",
                                              "LeftHand", "RightForeArm", "RightHand") for a in "XYZ"]


def load_clip_csv(name, csv_dir=CSV_DIR):
    """Runtime ingestion of the reference's 4-CSV clip format through the native loader (libhumenv.so,
    hum_clip_csv_parse: pandas' float converter, bit-identical tables; no pandas needed)."""
    import ctypes
    from . import _native as N
    L = N.lib()
    d, n = csv_dir.encode(), name.encode()
    sz = (ctypes.c_int32 * 4)()
    N.check(L.hum_clip_csv_sizes(d, n, sz), "hum_clip_csv_sizes")
    arrs = [np.zeros((sz[k], 27 if k == 3 else 14)) for k in range(4)]
    dp = ctypes.POINTER(ctypes.c_double)
    N.check(L.hum_clip_csv_parse(d, n, *[a.ctypes.data_as(dp) for a in arrs]), "hum_clip_csv_parse")
    return Clip(name, *arrs, list(JOINT_COLS), list(EP_COLS))
