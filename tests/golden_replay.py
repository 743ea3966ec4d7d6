"""Shared helpers: replay a golden scenario (tests/golden/make_golden.py) through an env implementation."""
import numpy as np

BOOK_SCALARS = ["frame", "cur_timestep", "highLevelDegTarget", "lowTargetScore", "deltaJoints", "deltaVelJoints",
                "bodyPostureScore", "electricityScore", "jointLimitScore", "aliveReward", "delta_lowTargetScore",
                "predefinedTargetIndex"]
BOOK_VECS = ["target", "starting_robot_pos", "robot_pos", "starting_ep_pos", "walk_target"]


def rec(g, name):
    pre = name + "/"
    return {k[len(pre):]: g[k] for k in g.files if k.startswith(pre)}


class ScriptedRNG:
    def __init__(self, draws):
        self.draws = [tuple(int(x) for x in d) for d in draws]
        self.i = 0

    def integers(self, lo, hi):
        elo, ehi, v = self.draws[self.i]
        assert (elo, ehi) == (lo, hi), ((elo, ehi), (lo, hi))
        self.i += 1
        return v
