#!/usr/bin/env python3
"""MJCF -> articulated-model compiler for the humanoid env.

Reads `humanoid_symmetric_2.xml` (reference: `/root/reference/humanoid_symmetric_2.xml`, loaded by
`humanoid.py:17-24` through pybullet's MJCF importer) and emits the tables the HIP kernel is compiled
against:

* `csrc/model_gen.h`      - constexpr tables (static tree => fully unrolled kernel, no indirect indexing)
* `data/humanoid_symmetric_2.model.json` - the same model as data (read by tests and the CPU oracle)

Model semantics (see DESIGN.md "Physics model"):

* Bodies whose MJCF <body> carries k>=1 hinge joints become one articulated body with a k-dof joint
  group (the k hinges composed intrinsically, in XML order).  This is exactly equivalent to pybullet's
  importer layout (k zero-mass dummy links `link0_N` chained by hinges, then a fixed joint to the body
  link), which is why the reference sees parts named `link0_11` (right-knee dummy) etc.
  (`low_level_env.py:139-144`, `Eksplor Ray RLLib.ipynb` cell 43).
* Bodies without joints (feet, hands) are rigidly merged into their parent (fixed joint).
* Each body frame has the MJCF body orientation and its origin at the joint pivot; the base (torso)
  frame origin is the torso centre of mass (pybullet's base frame is the inertial frame).
* Mass properties from geoms (`<compiler inertiafromgeom="true">`, density 1000): exact capsule
  (cylinder + hemispheres) and sphere inertias, combined with the parallel-axis theorem.
* The 33 "parts" whose mean x/y gives `body_xyz` (pybullet_envs WalkerBase.calc_state) are listed in
  pybullet's dict order: link COMs for body links, pivots for dummy links, plus the floor.

Usage:  python tools/mjcf_compile.py [--xml PATH]
"""
import argparse
import json
import math
import os
import xml.etree.ElementTree as ET

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
DEFAULT_XML = "/root/reference/humanoid_symmetric_2.xml"
DENSITY = 1000.0

# CustomHumanoidRobot motor table (humanoid.py:28-37): motor order and power; torque gain power=0.41 (:23)
MOTORS = [
    ("abdomen_z", 100), ("abdomen_y", 100), ("abdomen_x", 100),
    ("right_hip_x", 100), ("right_hip_z", 100), ("right_hip_y", 300), ("right_knee", 200),
    ("left_hip_x", 100), ("left_hip_z", 100), ("left_hip_y", 300), ("left_knee", 200),
    ("right_shoulder_x", 75), ("right_shoulder_y", 75), ("right_elbow", 75),
    ("left_shoulder_x", 75), ("left_shoulder_y", 75), ("left_elbow", 75),
]
POWER = 0.41


def _vec(s, n=3):
    v = [float(x) for x in s.split()]
    assert len(v) >= n, s
    return np.array(v[:n], dtype=np.float64)


def _quat_to_mat(q):
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def _geom_mass_props(g):
    """(mass, com, inertia-about-com) of one geom in its body's MJCF coordinates."""
    r = g["r"]
    if g["type"] == "sphere":
        m = DENSITY * 4.0 / 3.0 * math.pi * r ** 3
        return m, g["p1"].copy(), np.eye(3) * 0.4 * m * r * r
    a, b = g["p1"], g["p2"]
    L = float(np.linalg.norm(b - a))
    u = (b - a) / L
    mc = DENSITY * math.pi * r * r * L                      # cylinder
    mh = DENSITY * 2.0 / 3.0 * math.pi * r ** 3             # one hemisphere
    i_ax = 0.5 * mc * r * r + 2 * 0.4 * mh * r * r
    d = 0.5 * L + 3.0 * r / 8.0                             # hemisphere COM distance from centre
    i_perp = mc * (3 * r * r + L * L) / 12.0 + 2 * (83.0 / 320.0 * mh * r * r + mh * d * d)
    I = i_perp * (np.eye(3) - np.outer(u, u)) + i_ax * np.outer(u, u)
    return mc + 2 * mh, 0.5 * (a + b), I


def _combine(props):
    m = sum(p[0] for p in props)
    c = sum(p[0] * p[1] for p in props) / m
    I = np.zeros((3, 3))
    for mi, ci, Ii in props:
        dd = ci - c
        I += Ii + mi * (dd @ dd * np.eye(3) - np.outer(dd, dd))
    return m, c, I


def parse(xml_path):
    root = ET.parse(xml_path).getroot()
    comp = root.find("compiler")
    deg = comp is None or comp.get("angle", "degree") == "degree"
    dj = root.find("default/joint")
    def_damp = float(dj.get("damping", "0")) if dj is not None else 0.0
    def_arm = float(dj.get("armature", "0")) if dj is not None else 0.0

    mj_bodies = []  # flat list in XML (DFS) order

    def walk(el, parent):
        idx = len(mj_bodies)
        pos = _vec(el.get("pos", "0 0 0"))
        quat = _vec(el.get("quat", "1 0 0 0"), 4)
        geoms = []
        for g in el.findall("geom"):
            gt = g.get("type", "sphere")
            size = _vec(g.get("size"), 1)
            r = float(size[0])
            if g.get("fromto") is not None:
                ft = [float(x) for x in g.get("fromto").split()]
                p1, p2 = np.array(ft[:3]), np.array(ft[3:])
            else:
                p1 = p2 = _vec(g.get("pos", "0 0 0"))
            assert gt in ("sphere", "capsule"), gt
            geoms.append({"name": g.get("name"), "type": gt, "r": r, "p1": np.array(p1), "p2": np.array(p2)})
        joints = []
        for j in el.findall("joint"):
            assert j.get("type", "hinge") == "hinge"
            rng = _vec(j.get("range"), 2)
            if deg:
                rng = rng * math.pi / 180.0
            joints.append({
                "name": j.get("name"), "axis": _vec(j.get("axis", "0 0 1")), "pos": _vec(j.get("pos", "0 0 0")),
                "lo": float(rng[0]), "hi": float(rng[1]),
                "damping": float(j.get("damping", def_damp)), "armature": float(j.get("armature", def_arm)),
                "stiffness": float(j.get("stiffness", "0")),
            })
        mj_bodies.append({"name": el.get("name"), "parent": parent, "pos": pos, "quat": quat,
                          "R": _quat_to_mat(quat), "geoms": geoms, "joints": joints})
        for ch in el.findall("body"):
            walk(ch, idx)

    top = root.find("worldbody").findall("body")
    assert len(top) == 1
    walk(top[0], -1)
    return mj_bodies


def compile_model(xml_path):
    mj = parse(xml_path)
    # --- pybullet link naming (link0_<counter>; torso = 1) and parts order -------------------------
    counter = 1
    link_seq = []  # (link name, mj body index, kind) in creation order (excluding torso)
    for bi, b in enumerate(mj):
        if bi == 0:
            continue
        for j in b["joints"]:
            counter += 1
            link_seq.append(("link0_%d" % counter, bi, "dummy"))
        counter += 1
        link_seq.append((b["name"], bi, "body"))
    assert len(link_seq) == 31, len(link_seq)

    # --- articulated bodies: jointed MJCF bodies; jointless ones merge into the parent -------------
    art_of = {}      # mj index -> articulated body index
    bodies, dofs = [], []
    for bi, b in enumerate(mj):
        if bi == 0 or b["joints"]:
            piv = None
            if b["joints"]:
                piv = b["joints"][0]["pos"]
                for j in b["joints"]:
                    assert np.allclose(j["pos"], piv), "joint group must share a pivot"
            art_of[bi] = len(bodies)
            bodies.append({"name": b["name"], "mj": bi, "merged": [], "pivot": piv})
        else:
            pa = b["parent"]
            while pa not in art_of:
                pa = mj[pa]["parent"]
            bodies[art_of[pa]]["merged"].append(b["name"])

    # origin of each articulated frame in its MJCF body coordinates
    def own_geoms(bi):
        return [_geom_mass_props(g) for g in mj[bi]["geoms"]]

    torso_m, torso_c, _ = _combine(own_geoms(0))
    for ab in bodies:
        ab["origin_mj"] = torso_c if ab["mj"] == 0 else ab["pivot"]
    # mj body -> (articulated index, rotation, translation) mapping points in mj coords to art coords
    xf = {}
    for bi, b in enumerate(mj):
        if bi in art_of:
            ab = bodies[art_of[bi]]
            xf[bi] = (art_of[bi], np.eye(3), -ab["origin_mj"])
        else:
            pa, Rpa, tpa = xf[b["parent"]]
            # x_parentmj = R_b x + pos_b ; x_art = Rpa x_parentmj + tpa
            xf[bi] = (pa, Rpa @ b["R"], Rpa @ b["pos"] + tpa)

    def to_art(bi, p):
        _, Rm, tm = xf[bi]
        return Rm @ p + tm

    # geoms, mass props per articulated body
    geoms = []
    for bi, b in enumerate(mj):
        ai = xf[bi][0]
        for g in b["geoms"]:
            geoms.append({"name": g["name"], "body": ai, "type": 0 if g["type"] == "sphere" else 1, "r": g["r"],
                          "p1": to_art(bi, g["p1"]), "p2": to_art(bi, g["p2"]), "mj": bi})
    for ai, ab in enumerate(bodies):
        props = []
        for g in geoms:
            if g["body"] != ai:
                continue
            m, c, I = _geom_mass_props({"type": "sphere" if g["type"] == 0 else "capsule", "r": g["r"],
                                        "p1": g["p1"], "p2": g["p2"]})
            # geoms live in art coords already; inertia frame is the art frame (rotation Rm applied)
            props.append((m, c, I))
        m, c, I = _combine(props)
        ab["mass"], ab["com"], ab["inertia"] = m, c, I

    # kinematic offsets: parent art frame -> this art frame at q = 0
    for ai, ab in enumerate(bodies):
        bi = ab["mj"]
        if ai == 0:
            ab["parent"] = -1
            ab["R_off"] = np.eye(3)
            ab["t_off"] = np.zeros(3)
            continue
        pmj = mj[bi]["parent"]
        pa, Rp, tp = xf[pmj]
        ab["parent"] = pa
        # x_parentmj = R_b x_bmj + pos_b ; origin of this frame (pivot) in parent art coords
        ab["R_off"] = Rp @ mj[bi]["R"]
        ab["t_off"] = Rp @ (mj[bi]["R"] @ ab["pivot"] + mj[bi]["pos"]) + tp

    # dofs in XML order
    for ai, ab in enumerate(bodies):
        ab["dof0"] = len(dofs)
        ab["ndof"] = len(mj[ab["mj"]]["joints"])
        for j in mj[ab["mj"]]["joints"]:
            ax = j["axis"] / np.linalg.norm(j["axis"])
            nz = [k for k in range(3) if abs(ax[k]) > 1e-12]
            assert len(nz) == 1, "axis-aligned hinge axes expected"
            dofs.append({"name": j["name"], "body": ai, "axis": ax, "axis_index": nz[0],
                         "axis_sign": float(np.sign(ax[nz[0]])), "lo": j["lo"], "hi": j["hi"],
                         "damping": j["damping"], "armature": j["armature"], "stiffness": j["stiffness"]})
    assert len(dofs) == 17

    # parts in pybullet dict order: link0_2, torso, link0_3, lwaist, ..., floor
    def geoms_com_mj(bi):
        props = own_geoms(bi)
        return _combine(props)[1] if props else np.zeros(3)

    parts = []
    for k, (name, bi, kind) in enumerate(link_seq):
        ai = xf[bi][0]
        if kind == "dummy":
            p = np.zeros(3)  # pivot == articulated frame origin
        else:
            p = to_art(bi, geoms_com_mj(bi))
        parts.append({"name": name, "body": ai, "p": p})
        if k == 0:
            parts.append({"name": "torso", "body": 0, "p": np.zeros(3)})
    parts.append({"name": "floor", "body": -1, "p": np.zeros(3)})
    assert len(parts) == 33

    # self-collision pairs: different bodies, neither an ancestor of the other
    def ancestors(ai):
        out = set()
        while bodies[ai]["parent"] >= 0:
            ai = bodies[ai]["parent"]
            out.add(ai)
        return out

    pairs = []
    for ga in range(len(geoms)):
        for gb in range(ga + 1, len(geoms)):
            a, b = geoms[ga]["body"], geoms[gb]["body"]
            if a == b or a in ancestors(b) or b in ancestors(a):
                continue
            pairs.append([ga, gb])

    # mass-carrying pybullet links (body link + merged fixed children), each with its own mass properties
    # (Bullet's per-link velocity damping acts link by link, btMultiBody m_linearDamping/m_angularDamping)
    mlinks = []
    for bi, b in enumerate(mj):
        if not b["geoms"]:
            continue
        ai = xf[bi][0]
        props = [_geom_mass_props({"type": "sphere" if g["type"] == 0 else "capsule", "r": g["r"], "p1": g["p1"],
                                   "p2": g["p2"]}) for g in geoms if g["mj"] == bi]
        m, c, I = _combine(props)
        mlinks.append({"name": b["name"], "body": ai, "mass": m, "com": c, "inertia": I})

    dof_index = {d["name"]: i for i, d in enumerate(dofs)}
    actions = [{"name": n, "dof": dof_index[n], "power": p, "gain": POWER * p} for n, p in MOTORS]

    def fl(x):
        return [float(v) for v in np.asarray(x).ravel()]

    model = {
        "name": os.path.splitext(os.path.basename(xml_path))[0],
        "density": DENSITY,
        "bodies": [{"name": b["name"], "parent": b["parent"], "dof0": b["dof0"], "ndof": b["ndof"],
                    "R_off": fl(b["R_off"]), "t_off": fl(b["t_off"]), "mass": float(b["mass"]),
                    "com": fl(b["com"]), "inertia": fl(b["inertia"]), "merged": b["merged"]} for b in bodies],
        "dofs": [{"name": d["name"], "body": d["body"], "axis": fl(d["axis"]), "axis_index": d["axis_index"],
                  "axis_sign": d["axis_sign"], "lo": d["lo"], "hi": d["hi"], "damping": d["damping"],
                  "armature": d["armature"], "stiffness": d["stiffness"]} for d in dofs],
        "geoms": [{"name": g["name"], "body": g["body"], "type": g["type"], "r": g["r"],
                   "p1": fl(g["p1"]), "p2": fl(g["p2"])} for g in geoms],
        "parts": [{"name": p["name"], "body": p["body"], "p": fl(p["p"])} for p in parts],
        "pairs": pairs,
        "actions": actions,
        "links": [{"name": L["name"], "body": L["body"], "mass": float(L["mass"]), "com": fl(L["com"]),
                   "inertia": fl(L["inertia"])} for L in mlinks],
    }
    return model


def emit_header(model, path):
    B, D, G, P = model["bodies"], model["dofs"], model["geoms"], model["parts"]

    def arr(name, ctype, vals, fmt="{!r}"):
        return "inline constexpr %s %s[%d] = {%s};\n" % (ctype, name, len(vals), ", ".join(fmt.format(v) for v in vals))

    def darr(name, vals):
        return arr(name, "double", [float(v) for v in vals], "{!r}")

    s = []
    s.append("// GENERATED by tools/mjcf_compile.py from %s.xml - do not edit.\n" % model["name"])
    s.append("// Articulated humanoid model (see DESIGN.md 'Physics model'); all lengths in metres, SI units.\n")
    s.append("#pragma once\nnamespace hm {\n")
    s.append("inline constexpr int NB = %d, NDOF = %d, NGEOM = %d, NPART = %d, NPAIR = %d, NACT = %d;\n"
             % (len(B), len(D), len(G), len(P), len(model["pairs"]), len(model["actions"])))
    s.append(arr("body_parent", "int", [b["parent"] for b in B]))
    s.append(arr("body_dof0", "int", [b["dof0"] for b in B]))
    s.append(arr("body_ndof", "int", [b["ndof"] for b in B]))
    s.append(darr("body_Roff", [x for b in B for x in b["R_off"]]))
    s.append(darr("body_toff", [x for b in B for x in b["t_off"]]))
    s.append(darr("body_mass", [b["mass"] for b in B]))
    s.append(darr("body_com", [x for b in B for x in b["com"]]))
    s.append(darr("body_inertia", [x for b in B for x in b["inertia"]]))
    s.append(arr("dof_body", "int", [d["body"] for d in D]))
    s.append(arr("dof_axis", "int", [d["axis_index"] for d in D]))
    s.append(darr("dof_sign", [d["axis_sign"] for d in D]))
    s.append(darr("dof_lo", [d["lo"] for d in D]))
    s.append(darr("dof_hi", [d["hi"] for d in D]))
    s.append(darr("dof_damping", [d["damping"] for d in D]))
    s.append(arr("geom_body", "int", [g["body"] for g in G]))
    s.append(arr("geom_type", "int", [g["type"] for g in G]))
    s.append(darr("geom_r", [g["r"] for g in G]))
    s.append(darr("geom_p1", [x for g in G for x in g["p1"]]))
    s.append(darr("geom_p2", [x for g in G for x in g["p2"]]))
    s.append(arr("pair_a", "int", [p[0] for p in model["pairs"]]))
    s.append(arr("pair_b", "int", [p[1] for p in model["pairs"]]))
    s.append(arr("part_body", "int", [p["body"] for p in P]))
    s.append(darr("part_p", [x for p in P for x in p["p"]]))
    Lk = model["links"]
    s.append("inline constexpr int NLINK = %d;\n" % len(Lk))
    s.append(arr("link_body", "int", [L["body"] for L in Lk]))
    s.append(darr("link_mass", [L["mass"] for L in Lk]))
    s.append(darr("link_com", [x for L in Lk for x in L["com"]]))
    s.append(darr("link_inertia", [x for L in Lk for x in L["inertia"]]))
    s.append(arr("act_dof", "int", [a["dof"] for a in model["actions"]]))
    s.append(darr("act_gain", [a["gain"] for a in model["actions"]]))
    s.append("}  // namespace hm\n")
    with open(path, "w") as f:
        f.write("".join(s))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--xml", default=DEFAULT_XML)
    ap.add_argument("--out-json", default=os.path.join(PKG, "data", "humanoid_symmetric_2.model.json"))
    ap.add_argument("--out-header", default=os.path.join(PKG, "csrc", "model_gen.h"))
    a = ap.parse_args()
    model = compile_model(a.xml)
    with open(a.out_json, "w") as f:
        json.dump(model, f, indent=1)
    emit_header(model, a.out_header)
    tm = sum(b["mass"] for b in model["bodies"])
    print("bodies=%d dofs=%d geoms=%d parts=%d pairs=%d total_mass=%.4f kg"
          % (len(model["bodies"]), len(model["dofs"]), len(model["geoms"]), len(model["parts"]),
             len(model["pairs"]), tm))


if __name__ == "__main__":
    main()
