"""ORACLE - test infrastructure only (same rules as oracle/oracle.py: only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it, and only as the checker).

CPU restatement of the reference's two-level env `HierarchicalHumanoidEnv` (/root/reference/hier_env.py,
registered as "HumanoidBulletEnv-v0-Hier" by train_config.py:18-20,320), cited per method, plus
`math_util.projPointLineSegment` (math_util.py:20-27).  Physics, calc_state and the RNG are shared with
oracle/oracle.py.  Parity of the env logic is PINNED by tests/golden/golden_hier.npz, produced by importing the
real hier_env.py under stubs (tests/golden/make_golden_hier.py); physics parity vs PyBullet is unpinned.
"""
import numpy as np
from scipy.spatial.transform import Rotation as R

import oracle as O

HIGH, LOW = "high_level_agent", "low_level_agent"


def proj_point_line_segment(point, lineStart, lineEnd):   # math_util.py:20-27
    lineVec = lineEnd - lineStart
    lineLen = np.linalg.norm(lineVec)
    t = np.dot(point - lineStart, lineVec) / np.square(lineLen)
    t = np.clip(t, 0, 1)
    return lineStart + t * lineVec


class OracleHierEnv:
    """Single-lane restatement of HierarchicalHumanoidEnv (hier_env.py:38-641).  `clip` is the selected motion
    (motion_list[selected_motion] = motion09_03, hier_env.py:50,179)."""

    def __init__(self, clip, seed=0, lane=0, params=None, rng=None, numpy_semantics=O.DEFAULT_NUMPY,
                 phys_precision="fp64"):
        self.clip = clip
        self.params = params
        self.phys_precision = phys_precision   # "fp32": physics through the float instantiation (O.phys_step)
        self.numpy_semantics = numpy_semantics
        self.step_per_level = 5                                     # :58
        self.steps_remaining_at_level = self.step_per_level
        self.num_high_level_steps = 0
        self.cur_timestep = 0
        self.max_timestep = 3000                                    # :83
        self.max_frame = clip.pos.shape[0] - 1                      # :87
        self.rng = rng if rng is not None else O.LaneRNG(seed, lane)   # :89 (explicit, counter based)
        self.joint_weight_sum = sum(O.JOINT_WEIGHT.values())
        self.joint_vel_weight_sum = sum(O.JOINT_VEL_WEIGHT.values())
        self.target = np.array([1, 0, 0])                           # :159
        self.targetLen = 5
        self.highLevelDegTarget = 0
        self.predefinedTarget = np.array([[]])
        self.predefinedTargetIndex = 0
        self.usePredefinedTarget = False
        self.skipFrame = 2                                          # :167
        self.selected_motion_frame = 0
        self.starting_ep_pos = np.array([0, 0, 0])                  # :173 (persists across resets)
        self.starting_robot_pos = np.array([0, 0, 0])
        self.robot_pos = np.array([0, 0, 0])
        self.walk_target = (1e3, 0.0)
        self.state = np.zeros(O.NSTATE)
        self.state[6] = 1.0
        self.body_xyz = (0.0, 0.0, 0.0)
        self.cur_obs = np.zeros(42, dtype=np.float32)
        self.initReward()

    @classmethod
    def from_lane(cls, clip, phys, book, bk, numpy_semantics=O.DEFAULT_NUMPY, phys_precision="fp64"):
        """An env holding exactly one product lane's state (hum_get_state rows; bk = the HUM_BK_* column map, passed
        in: the oracle imports nothing from the product).  cur_obs is the calc_state of that state under the lane's
        walk target, which is what the reference holds between calls (its walk target changes only in
        high_level_step and resetFromFrame, after which cur_obs is not recomputed until the next low step)."""
        o = cls(clip, numpy_semantics=numpy_semantics, phys_precision=phys_precision)
        o.state = np.array(phys, dtype=np.float64).copy()
        o.selected_motion_frame = int(book[bk["frame"]])
        o.cur_timestep = int(book[bk["cur_timestep"]])
        o.predefinedTargetIndex = int(book[bk["predefinedTargetIndex"]])
        for k in ("target", "starting_robot_pos", "robot_pos", "starting_ep_pos"):
            setattr(o, k, np.array(book[bk[k]:bk[k] + 3], dtype=np.float64))
        o.walk_target = (float(book[bk["walk_target"]]), float(book[bk["walk_target"] + 1]))
        o.highLevelDegTarget = float(book[bk["highLevelDegTarget"]])
        for k in ("lowTargetScore", "deltaJoints", "deltaVelJoints", "bodyPostureScore", "electricityScore",
                  "jointLimitScore", "aliveReward", "delta_lowTargetScore", "highTargetScore", "driftScore",
                  "cumulative_driftScore", "delta_highTargetScore", "cumulative_aliveReward"):
            setattr(o, k, float(book[bk[k]]))
        o.steps_remaining_at_level = int(book[bk["steps_remaining_at_level"]])
        o.num_high_level_steps = int(book[bk["num_high_level_steps"]])
        o.body_xyz = (float(book[bk["body_xy"]]), float(book[bk["body_xy"] + 1]), float(phys[2]))
        key = int(book[bk["rng_key_lo"]]) | (int(book[bk["rng_key_hi"]]) << 32)
        o.rng = O.LaneRNG(key=key, counter=int(book[bk["rng_counter"]]))
        obs, _, js, jal, _ = O.calc_state(o.state, o.walk_target)
        o.cur_obs, o.joint_speeds, o.joints_at_limit = obs, js, jal
        return o

    def initReward(self):                                           # :183-206
        self.deltaJoints = 0
        self.deltaVelJoints = 0
        self.deltaEndPoints = 0
        self.baseReward = 0
        self.lowTargetScore = 0
        self.aliveReward = 0
        self.electricityScore = 0
        self.jointLimitScore = 0
        self.bodyPostureScore = 0
        self.highTargetScore = -self.targetLen
        self.driftScore = 0
        self.cumulative_driftScore = 0
        self.delta_deltaJoints = 0
        self.delta_deltaVelJoints = 0
        self.delta_deltaEndPoints = 0
        self.delta_lowTargetScore = 0
        self.delta_bodyPostureScore = 0
        self.delta_highTargetScore = 0
        self.cumulative_aliveReward = 0

    # -- flat env stand-ins ------------------------------------------------------------------------------
    def _calc_state(self):
        obs, body_xyz, js, jal, rpy = O.calc_state(self.state, self.walk_target)
        self.body_xyz, self.joint_speeds, self.joints_at_limit = body_xyz, js, jal
        return obs

    def rpy_now(self):
        return O.euler_from_quaternion(self.state[3:7])

    def setJointsOrientation(self, frame_idx):                      # :214-225
        c = self.clip
        for name in ("abdomen_x", "abdomen_y", "abdomen_z"):
            d = O.DOF_NAMES.index(name)
            self.state[13 + d] = 0
            self.state[30 + d] = 0
        for joint, col in O.JOINT_MAP:
            d = O.DOF_NAMES.index(joint)
            self.state[13 + d] = c.pos[frame_idx, c.jcol(col)]
            self.state[30 + d] = c.vel[frame_idx, c.jcol(col)]

    def incFrame(self, inc):                                        # :227-233
        self.selected_motion_frame = (self.selected_motion_frame + inc) % (self.max_frame - 1)
        if self.selected_motion_frame == 0:
            self.starting_ep_pos = self.robot_pos.copy()

    def reset(self):                                                # :235-243
        return self.resetFromFrame(startFrame=self.rng.integers(0, self.max_frame - 5),
                                   resetYaw=self.rng.integers(-180, 180), startFromRef=True, initVel=True)

    def setWalkTarget(self, x, y):                                  # :245-249
        self.walk_target = (x, y)

    def getRandomVec(self, vecLen, z, initYaw=0):                   # :251-257
        randomRad = initYaw + np.deg2rad(self.rng.integers(-180, 180))
        return np.array([np.cos(randomRad) * vecLen, np.sin(randomRad) * vecLen, z])

    def resetFromFrame(self, startFrame=0, resetYaw=0, startFromRef=True, initVel=True):   # :259-319
        self.state[:] = 0
        self.state[6] = 1.0
        if not startFromRef:
            self.state[13:30] = self.rng.joint_noise()
        self.cur_timestep = 0
        if self.usePredefinedTarget:
            self.predefinedTargetIndex = 0
            self.target = self.predefinedTarget[self.predefinedTargetIndex].copy()
        else:
            self.target = self.getRandomVec(self.targetLen, 0)
        self.setWalkTarget(self.target[0], self.target[1])
        if startFromRef:
            self.selected_motion_frame = startFrame
            self.setJointsOrientation(self.selected_motion_frame)
        robotPos = np.array([0, 0, 1.17])
        self.robot_pos = np.array([robotPos[0], robotPos[1], 0])
        self.last_robotPos = self.robot_pos.copy()
        self.starting_robot_pos = self.robot_pos.copy()
        self.state[0:3] = robotPos
        degToTarget = np.rad2deg(np.arctan2(self.target[1], self.target[0])) + resetYaw
        self.setWalkTarget(np.cos(degToTarget) * 1000, np.sin(degToTarget) * 1000)
        robotRot = R.from_euler("z", degToTarget, degrees=True)
        self.state[3:7] = robotRot.as_quat()
        self.highLevelDegTarget = np.deg2rad(degToTarget)
        f = self.selected_motion_frame
        rotDeg = R.from_euler("z", degToTarget, degrees=True)
        if startFromRef and initVel:
            rightLegPosRef = rotDeg.apply(O.get_joint_pos(self.clip, f, "RightLeg"))
            rightLegPosRefNext = rotDeg.apply(O.get_joint_pos(self.clip, f + 1, "RightLeg"))
            startingVelocity = (rightLegPosRefNext - rightLegPosRef) / 0.0165
            self.state[7:10] = startingVelocity
            self.state[10:13] = 0
        self.initReward()
        self.steps_remaining_at_level = self.step_per_level
        self.num_high_level_steps = 0
        self.frame_update_cnt = 0
        self.incFrame(self.skipFrame)
        self.cur_obs = self._calc_state()
        return {HIGH: self.getHighLevelObs()}

    def getLowLevelObs(self):                                       # :321-334
        c = self.clip
        jt = []
        for _, col in O.JOINT_MAP:
            jt.append(c.rel[self.selected_motion_frame, c.jcol(col)])
            jt.append(c.vel[self.selected_motion_frame, c.jcol(col)])
        return np.hstack((self.cur_obs, np.array(jt)))

    def getHighLevelObs(self):                                      # :336-353
        _, _, yaw = self.rpy_now()
        targetTheta = np.arctan2(self.target[1] - self.robot_pos[1], self.target[0] - self.robot_pos[0])
        angleToTarget = targetTheta - yaw
        degTarget = [np.cos(angleToTarget), np.sin(angleToTarget)]
        startPosTheta = np.arctan2(self.starting_robot_pos[1] - self.robot_pos[1],
                                   self.starting_robot_pos[0] - self.robot_pos[0])
        angleToStart = startPosTheta - yaw
        degStart = [np.cos(angleToStart), np.sin(angleToStart)]
        return np.hstack((self.cur_obs[:1], degTarget, degStart, self.cur_obs[3:]))

    def step(self, action_dict, debug=False, physics=True):         # :355-366
        assert len(action_dict) == 1, action_dict
        self.robot_pos[0] = self.body_xyz[0]
        self.robot_pos[1] = self.body_xyz[1]
        self.robot_pos[2] = 0
        if HIGH in action_dict:
            return self.high_level_step(action_dict[HIGH], debug=debug)
        return self.low_level_step(list(action_dict.values())[0], debug=debug, physics=physics)

    def calcJointScore(self):                                       # :368-386 (useExp=True)
        c, d = self.clip, 0
        for jm, col in O.JOINT_MAP:
            d += np.abs(self.state[13 + O.DOF_NAMES.index(jm)] - c.pos[self.selected_motion_frame, c.jcol(col)]) \
                * O.JOINT_WEIGHT[jm]
        return np.exp(4 * (-d / self.joint_weight_sum))

    def calcJointVelScore(self):                                    # :388-406 (useExp=True)
        c, d = self.clip, 0
        for jm, col in O.JOINT_MAP:
            d += np.abs(self.state[30 + O.DOF_NAMES.index(jm)] - c.vel[self.selected_motion_frame, c.jcol(col)]) \
                * O.JOINT_VEL_WEIGHT[jm]
        return np.exp((-d / self.joint_vel_weight_sum) / 2)

    def calcHighLevelTargetScore(self):                             # :432-434
        return -np.linalg.norm(self.target - self.robot_pos)

    def calcLowLevelTargetScore(self):                              # :436-437
        return 0

    def calcBodyPostureScore(self):                                 # :439-444 (useExp=True)
        roll, pitch, yaw = self.rpy_now()
        return np.exp(-(np.abs(yaw - self.highLevelDegTarget) + np.abs(roll) + np.abs(pitch)))

    def calcAliveReward(self):                                      # :446-449
        z = self.cur_obs[0] + 0.8
        if self.numpy_semantics == O.NUMPY_1:
            z = float(self.cur_obs[0]) + 0.8
        return +2 if z > 0.75 else -1

    def calcElectricityCost(self, action):                          # :451-456
        runningCost = -1.0 * float(np.abs(action * self.joint_speeds).mean())
        stallCost = -0.1 * float(np.square(action).mean())
        return runningCost + stallCost

    def calcJointLimitCost(self):                                   # :458-459
        return -0.1 * self.joints_at_limit

    def calcDriftScore(self):                                       # :461-467
        projection = proj_point_line_segment(self.robot_pos, self.starting_robot_pos, self.target)
        score = np.linalg.norm(projection - self.robot_pos)
        return np.exp(-6 * score)

    def checkTarget(self):                                          # :469-487
        distToTarget = np.linalg.norm(self.robot_pos - self.target)
        if distToTarget <= 0.5:
            _, _, yaw = self.rpy_now()
            randomTarget = self.getRandomVec(self.targetLen, 0, initYaw=yaw)
            newTarget = self.robot_pos + randomTarget
            if self.usePredefinedTarget:
                self.predefinedTargetIndex = (self.predefinedTargetIndex + 1) % len(self.predefinedTarget)
                newTarget = self.predefinedTarget[self.predefinedTargetIndex]
            self.starting_robot_pos = self.target.copy()
            self.target = newTarget
            self.highTargetScore = -np.linalg.norm(self.target - self.starting_robot_pos)

    def updateReward(self, action):                                 # :494-522
        jointScore = self.calcJointScore()
        jointVelScore = self.calcJointVelScore()
        lowTargetScore = self.calcLowLevelTargetScore()
        bodyPostureScore = self.calcBodyPostureScore()
        self.delta_deltaJoints = (jointScore - self.deltaJoints) / 0.0165
        self.delta_deltaVelJoints = (jointVelScore - self.deltaVelJoints) / 0.0165 * 0.1
        self.delta_lowTargetScore = (lowTargetScore - self.lowTargetScore) / 0.0165 * 0.1
        self.delta_bodyPostureScore = (bodyPostureScore - self.bodyPostureScore) / 0.0165 * 0.1
        self.deltaJoints = jointScore
        self.deltaVelJoints = jointVelScore
        self.lowTargetScore = lowTargetScore
        self.electricityScore = self.calcElectricityCost(action)
        self.jointLimitScore = self.calcJointLimitCost()
        self.aliveReward = self.calcAliveReward()
        self.cumulative_aliveReward += self.aliveReward
        self.bodyPostureScore = bodyPostureScore
        self.cumulative_driftScore += self.calcDriftScore()

    def updateRewardHigh(self):                                     # :524-536
        highTargetScore = self.calcHighLevelTargetScore()
        self.delta_highTargetScore = (highTargetScore - self.highTargetScore) / 0.0165
        self.delta_highTargetScore /= (self.step_per_level - self.steps_remaining_at_level + 1)
        self.highTargetScore = highTargetScore
        self.driftScore = self.cumulative_driftScore / (self.step_per_level - self.steps_remaining_at_level + 1)
        self.cumulative_driftScore = 0

    def high_level_step(self, action, debug=False):                 # :538-571
        actionDegree = np.rad2deg(np.arctan2(action[1], action[0]))
        _, _, yaw = self.rpy_now()
        newDegree = actionDegree + np.rad2deg(yaw)
        self.highLevelDegTarget = np.deg2rad(newDegree)
        cosTarget, sinTarget = np.cos(self.highLevelDegTarget), np.sin(self.highLevelDegTarget)
        newWalkTarget = self.robot_pos + np.array([cosTarget, sinTarget, 0]) * 5
        self.setWalkTarget(newWalkTarget[0], newWalkTarget[1])
        vRobotTarget = newWalkTarget - self.robot_pos
        lenSEP = np.linalg.norm(self.starting_ep_pos - self.robot_pos)
        self.starting_ep_pos = -vRobotTarget / np.linalg.norm(vRobotTarget)
        self.starting_ep_pos *= lenSEP
        self.starting_ep_pos += self.robot_pos
        self.steps_remaining_at_level = self.step_per_level
        self.num_high_level_steps += 1
        return {LOW: self.getLowLevelObs()}, {LOW: 0}, {"__all__": False}, {}

    def checkIfDone(self, debug=False):                             # :573-581
        isAlive = self.aliveReward > 0
        isNearTarget = np.linalg.norm(self.target - self.robot_pos) <= \
            np.linalg.norm(self.target - self.starting_robot_pos) + 1
        return (not isAlive) if debug else (not (isAlive and isNearTarget))

    def low_level_step(self, action, debug=False, physics=True):    # :583-641
        action = np.asarray(action, dtype=np.float32)
        self.steps_remaining_at_level -= 1
        if physics:
            self.state = O.phys_step(self.state, O.motor_torques(action, self.numpy_semantics), self.params,
                                     self.phys_precision)
        self.cur_obs = self._calc_state()
        self.updateReward(action=action)
        reward = [self.deltaJoints, self.deltaVelJoints, self.delta_lowTargetScore, self.electricityScore,
                  self.jointLimitScore, self.aliveReward, self.bodyPostureScore]
        totalReward = 0
        for r, w in zip(reward, O.REWARD_WEIGHT):
            totalReward += r * w
        self.incFrame(self.skipFrame)
        self.checkTarget()
        rew, obs = dict(), dict()
        done = {"__all__": False}
        f_done = self.checkIfDone(debug=debug)
        self.cur_timestep += 1
        if f_done or (self.cur_timestep >= self.max_timestep):
            self.updateRewardHigh()
            done["__all__"] = True
            rew[HIGH] = self.delta_highTargetScore * 0.3 + self.driftScore * 0.7
            obs[HIGH] = self.getHighLevelObs()
            obs[LOW] = self.getLowLevelObs()
            rew[LOW] = totalReward
            self.cumulative_aliveReward = 0
        elif self.steps_remaining_at_level <= 0:
            self.updateRewardHigh()
            rew[HIGH] = self.delta_highTargetScore * 0.3 + self.driftScore * 0.7
            obs[HIGH] = self.getHighLevelObs()
            self.cumulative_aliveReward = 0
        else:
            obs = {LOW: self.getLowLevelObs()}
            rew = {LOW: totalReward}
        return obs, rew, done, {}
