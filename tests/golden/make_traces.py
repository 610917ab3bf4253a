#!/usr/bin/env python3
"""Physics-free full-step traces from the reference task classes.

Run in the build container only (needs /root/reference):

    python tests/golden/make_traces.py

The reference ``Ant`` / ``Humanoid`` / ``Cartpole`` classes are constructed on
top of a fake ``gym`` object (SURVEY.md §8(c) "Full-step oracle", Appendix D):
``simulate`` overwrites the sim state with a seeded "physics output" that the
trace records, ``set_*_indexed`` copy rows into the sim buffers immediately and
``refresh_*`` are no-ops.  ``VecTask.step`` (vec_task.py:362-410) then runs the
reference's own ordering: action clamp -> pre_physics_step -> simulate ->
post_physics_step (progress += 1, reset_idx on the previous step's reset_buf,
compute_observations, compute_reward) -> timeout_buf -> obs clamp.

Every reset-noise draw the reference makes with the global torch RNG is
recorded as raw U(0,1) samples scattered to per-env rows, so the build's task
layer can replay the exact same resets from injected noise.

ShadowHand (tasks/shadow_hand.py) runs on the same fake gym extended with the
asset queries its constructor makes (tendons, actuators, DOF properties, global
actor indices); its reset draws are recorded per env as [goal-only 4 | reset_idx
53 | reset_target_pose 4] columns, and the state right before ``simulate`` (after
pre_physics_step's resets and PD targets) is recorded as well.

Output: tests/golden/trace_{ant,humanoid,cartpole,shadowhand}.npz
"""
import math
import os
import sys

import numpy as np
import torch
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refshim  # noqa: E402

_refshim.install()
from isaacgym import gymapi  # noqa: E402
from isaacgymenvs.utils import torch_jit_utils as tju  # noqa: E402

REF = _refshim.REF


class _Prop:
    def __init__(self, **k):
        self.__dict__.update(k)


class FakeGym:
    """Physics-free stand-in for isaacgym.gymapi.Gym (Appendix D surface)."""

    def __init__(self, spec, num_envs):
        self.spec = spec
        self.N = num_envs
        nd = spec["num_dof"]
        self.root = torch.zeros(num_envs * spec.get("actors", 1), 13)
        self.root[:, 2] = spec.get("start_z", 0.0)
        self.root[:, 6] = 1.0
        self.dof = torch.zeros(num_envs * nd, 2)
        self.sensors = torch.zeros(num_envs * spec.get("sensors", 0), 6)
        self.dof_force = torch.zeros(num_envs * nd)
        self.calls = []
        self.inject = None

    # --- setup --------------------------------------------------------------------------
    def create_sim(self, *a):
        return "sim"

    def add_ground(self, *a):
        pass

    def load_asset(self, *a):
        return "asset"

    def get_asset_dof_count(self, a):
        return self.spec["num_dof"]

    def get_asset_rigid_body_count(self, a):
        return len(self.spec["bodies"])

    def get_asset_joint_count(self, a):
        return self.spec["num_dof"]

    def get_asset_rigid_body_name(self, a, i):
        return self.spec["bodies"][i]

    def find_asset_rigid_body_index(self, a, name):
        return self.spec["bodies"].index(name)

    def get_asset_actuator_properties(self, a):
        return [_Prop(motor_effort=g) for g in self.spec["gears"]]

    def create_asset_force_sensor(self, *a):
        return 0

    def create_env(self, *a):
        return "env"

    def create_actor(self, *a):
        return 0

    def set_rigid_body_color(self, *a):
        pass

    def enable_actor_dof_force_sensors(self, *a):
        pass

    def get_actor_dof_properties(self, env, h):
        nd = self.spec["num_dof"]
        return {"lower": np.array(self.spec.get("lower", [0.0] * nd), dtype=np.float32),
                "upper": np.array(self.spec.get("upper", [0.0] * nd), dtype=np.float32),
                "driveMode": np.zeros(nd, dtype=np.int32),
                "stiffness": np.zeros(nd, dtype=np.float32),
                "damping": np.zeros(nd, dtype=np.float32)}

    def set_actor_dof_properties(self, *a):
        pass

    def find_actor_rigid_body_handle(self, env, h, name):
        return self.spec["bodies"].index(name)

    def prepare_sim(self, sim):
        pass

    # --- tensors ------------------------------------------------------------------------
    def acquire_actor_root_state_tensor(self, sim):
        return self.root

    def acquire_dof_state_tensor(self, sim):
        return self.dof

    def acquire_force_sensor_tensor(self, sim):
        return self.sensors

    def acquire_dof_force_tensor(self, sim):
        return self.dof_force

    def refresh_dof_state_tensor(self, sim):
        pass

    refresh_actor_root_state_tensor = refresh_force_sensor_tensor = refresh_dof_force_tensor = refresh_dof_state_tensor

    def set_dof_actuation_force_tensor(self, sim, t):
        self.calls.append(("actuation", t.clone()))

    def set_actor_root_state_tensor_indexed(self, sim, data, idx, n):
        idx = idx.long()
        self.root[idx] = data[idx]
        self.calls.append(("root_indexed", idx.clone()))

    def set_dof_state_tensor_indexed(self, sim, data, idx, n):
        nd = self.spec["num_dof"]
        idx = idx.long()
        d = data.view(self.N, nd, 2)
        self.dof.view(self.N, nd, 2)[idx] = d[idx]
        self.calls.append(("dof_indexed", idx.clone()))

    def simulate(self, sim):
        if self.inject is not None:
            root, dof, sens, dforce = self.inject
            self.root.copy_(root)
            self.dof.copy_(dof)
            if sens is not None:
                self.sensors.copy_(sens)
            if dforce is not None:
                self.dof_force.copy_(dforce)

    def fetch_results(self, *a):
        pass


def install_fake(fake):
    from isaacgym import gymtorch
    gymapi.acquire_gym = lambda: fake
    gymtorch.wrap_tensor = lambda t: t
    gymtorch.unwrap_tensor = lambda t: t


def load_task_cfg(name, num_envs, episode_length=None):
    with open(os.path.join(REF, "isaacgymenvs/cfg/task", name + ".yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["physics_engine"] = "physx"
    cfg["env"]["numEnvs"] = num_envs
    if episode_length is not None:
        cfg["env"]["episodeLength"] = episode_length
    cfg["sim"]["use_gpu_pipeline"] = False
    cfg["sim"]["physx"] = {}
    return cfg


class RandRecorder:
    """Wraps the task module's ``torch_rand_float`` so each draw's raw U(0,1) is kept."""

    def __init__(self):
        self.draws = []

    def __call__(self, lower, upper, shape, device):
        u = torch.rand(*shape, device=device)
        self.draws.append(u.clone())
        return (upper - lower) * u + lower


def physics_output(g, N, nd, lo, hi, z_range, nsens):
    root = torch.zeros(N, 13)
    root[:, 0:2] = torch.randn(N, 2, generator=g)
    root[:, 2] = z_range[0] + (z_range[1] - z_range[0]) * torch.rand(N, generator=g)
    yaw = (torch.rand(N, generator=g) * 2 - 1) * math.pi
    rp = (torch.rand(N, 2, generator=g) * 2 - 1) * 0.5
    root[:, 3:7] = tju.quat_from_euler_xyz(rp[:, 0], rp[:, 1], yaw)
    root[:, 7:13] = torch.randn(N, 6, generator=g)
    pos = lo + (hi - lo) * (torch.rand(N, nd, generator=g) * 1.1 - 0.05)
    vel = torch.randn(N, nd, generator=g) * 3
    dof = torch.stack([pos, vel], dim=-1).reshape(N * nd, 2)
    sens = torch.randn(N * nsens, 6, generator=g) * 10 if nsens else None
    return root, dof, sens


def run_locomotion(task, N=64, T=8, ep_len=5, reset_done=False):
    """reset_done=True: after every step the trace calls the reference's own ``VecTask.reset_done``
    (vec_task.py:442-457), the rl_games AMP agent/player pattern (learning/common_agent.py:458-459,
    common_player.py:173-174), and records its draws, the state it leaves and the observations it returns."""
    import importlib
    mod = importlib.import_module("isaacgymenvs.tasks." + task.lower())
    if task == "Ant":
        d = math.pi / 180
        spec = dict(num_dof=8, sensors=4, start_z=0.44, gears=[15.0] * 8,
                    bodies=["torso", "front_left_leg", "front_left_foot", "front_right_leg", "front_right_foot",
                            "left_back_leg", "left_back_foot", "right_back_leg", "right_back_foot"],
                    lower=[x * d for x in [-40, 30, -40, -100, -40, -100, -40, 30]],
                    upper=[x * d for x in [40, 100, 40, -30, 40, -30, 40, 100]])
        z_range, nsens, cls = (0.25, 0.7), 4, mod.Ant
    else:
        d = math.pi / 180
        deg = [(-45, 45), (-75, 30), (-35, 35), (-45, 15), (-60, 35), (-120, 45), (-160, 2), (-50, 50), (-50, 50),
               (-45, 15), (-60, 35), (-120, 45), (-160, 2), (-50, 50), (-50, 50), (-90, 70), (-90, 70), (-90, 50),
               (-90, 70), (-90, 70), (-90, 50)]
        spec = dict(num_dof=21, sensors=2, start_z=1.34,
                    gears=[67.5, 67.5, 67.5, 45, 45, 135, 90, 22.5, 22.5, 45, 45, 135, 90, 22.5, 22.5,
                           67.5, 67.5, 45, 67.5, 67.5, 45],
                    bodies=["torso", "head", "lower_waist", "pelvis", "right_thigh", "right_shin", "right_foot",
                            "left_thigh", "left_shin", "left_foot", "right_upper_arm", "right_lower_arm",
                            "right_hand", "left_upper_arm", "left_lower_arm", "left_hand"],
                    lower=[a * d for a, _ in deg], upper=[b * d for _, b in deg])
        z_range, nsens, cls = (0.7, 1.4), 2, mod.Humanoid
    fake = FakeGym(spec, N)
    install_fake(fake)
    rec = RandRecorder()
    mod.torch_rand_float = rec
    cfg = load_task_cfg(task, N, ep_len)
    torch.manual_seed(0)
    env = cls(cfg, "cpu", "cpu", -1, True, False, False)
    nd = spec["num_dof"]
    lo = torch.tensor(spec["lower"])
    hi = torch.tensor(spec["upper"])
    lo, hi = torch.minimum(lo, hi), torch.maximum(lo, hi)
    g = torch.Generator().manual_seed(1)
    out = {k: [] for k in ("actions", "phys_root", "phys_dof", "phys_sensors", "phys_dof_force", "noise",
                           "reset_mask", "obs", "rew", "reset", "progress", "timeouts", "potentials",
                           "prev_potentials", "root_after", "dof_after", "reset_in", "progress_in")}
    if reset_done:
        for k in ("rd_mask", "rd_noise", "rd_root", "rd_dof", "rd_reset", "rd_progress", "rd_potentials",
                  "rd_prev_potentials", "rd_obs"):
            out[k] = []
    out["init_obs"] = env.reset()["obs"].clone()
    for t in range(T):
        actions = torch.rand(N, env.num_actions, generator=g) * 2.4 - 1.2  # exercises the ±1 clip
        root, dof, sens = physics_output(g, N, nd, lo, hi, z_range, nsens)
        dforce = torch.randn(N * nd, generator=g) * 20 if task == "Humanoid" else None
        fake.inject = (root, dof, sens, dforce)
        reset_in = env.reset_buf.clone()
        progress_in = env.progress_buf.clone()
        rec.draws.clear()
        obs_dict, rew, reset, extras = env.step(actions)
        ids = reset_in.nonzero(as_tuple=False).flatten()
        noise = torch.zeros(N, 2 * nd)
        if len(ids) > 0:
            noise[ids, :nd] = rec.draws[0]
            noise[ids, nd:] = rec.draws[1]
        mask = torch.zeros(N, dtype=torch.int64)
        mask[ids] = 1
        out["actions"].append(actions)
        out["phys_root"].append(root)
        out["phys_dof"].append(dof.view(N, nd, 2))
        out["phys_sensors"].append(sens.view(N, nsens * 6))
        out["phys_dof_force"].append(dforce.view(N, nd) if dforce is not None else torch.zeros(N, nd))
        out["noise"].append(noise)
        out["reset_mask"].append(mask)
        out["obs"].append(obs_dict["obs"].clone())
        out["rew"].append(rew.clone())
        out["reset"].append(reset.clone())
        out["progress"].append(env.progress_buf.clone())
        out["timeouts"].append(extras["time_outs"].clone().long())
        out["potentials"].append(env.potentials.clone())
        out["prev_potentials"].append(env.prev_potentials.clone())
        out["root_after"].append(env.root_states.clone())
        out["dof_after"].append(env.dof_state.view(N, nd, 2).clone())
        out["reset_in"].append(reset_in)
        out["progress_in"].append(progress_in)
        if reset_done:
            done_in = env.reset_buf.clone()
            rec.draws.clear()
            rd_obs, rd_ids = env.reset_done()
            ids = done_in.nonzero(as_tuple=False).flatten()
            assert torch.equal(rd_ids, ids)
            noise = torch.zeros(N, 2 * nd)
            if len(ids) > 0:
                noise[ids, :nd] = rec.draws[0]
                noise[ids, nd:] = rec.draws[1]
            else:
                assert not rec.draws
            mask = torch.zeros(N, dtype=torch.int64)
            mask[ids] = 1
            out["rd_mask"].append(mask)
            out["rd_noise"].append(noise)
            out["rd_root"].append(env.root_states.clone())
            out["rd_dof"].append(env.dof_state.view(N, nd, 2).clone())
            out["rd_reset"].append(env.reset_buf.clone())
            out["rd_progress"].append(env.progress_buf.clone())
            out["rd_potentials"].append(env.potentials.clone())
            out["rd_prev_potentials"].append(env.prev_potentials.clone())
            out["rd_obs"].append(rd_obs["obs"].clone())
    res = {k: (torch.stack(v) if isinstance(v, list) else v) for k, v in out.items()}
    res["lower"], res["upper"] = lo, hi
    res["episode_length"] = torch.tensor(ep_len)
    return res


def run_cartpole(N=64, T=12):
    import importlib
    mod = importlib.import_module("isaacgymenvs.tasks.cartpole")
    spec = dict(num_dof=2, sensors=0, gears=[], bodies=["slider", "cart", "pole"])
    fake = FakeGym(spec, N)
    install_fake(fake)
    draws = []

    class _TorchProxy:
        def __getattr__(self, k):
            return getattr(torch, k)

        def rand(self, *shape, **kw):
            u = torch.rand(*shape, **kw)
            draws.append(u.clone())
            return u

    mod.torch = _TorchProxy()
    cfg = load_task_cfg("Cartpole", N)
    torch.manual_seed(0)
    env = mod.Cartpole(cfg, "cpu", "cpu", -1, True, False, False)
    g = torch.Generator().manual_seed(2)
    keys = ("actions", "phys_dof", "noise", "reset_mask", "obs", "rew", "reset", "progress", "timeouts",
            "dof_after", "reset_in", "progress_in", "actuation")
    out = {k: [] for k in keys}
    for t in range(T):
        actions = torch.rand(N, 1, generator=g) * 2.4 - 1.2
        dof = torch.randn(N, 2, 2, generator=g) * torch.tensor([[[2.0, 1.0], [1.0, 2.0]]])
        fake.inject = (fake.root, dof.reshape(N * 2, 2), None, None)
        reset_in = env.reset_buf.clone()
        progress_in = env.progress_buf.clone()
        draws.clear()
        fake.calls.clear()
        obs_dict, rew, reset, extras = env.step(actions)
        ids = reset_in.nonzero(as_tuple=False).flatten()
        noise = torch.zeros(N, 4)
        if len(ids) > 0:
            noise[ids, :2] = draws[0]
            noise[ids, 2:] = draws[1]
        mask = torch.zeros(N, dtype=torch.int64)
        mask[ids] = 1
        act = [c[1] for c in fake.calls if c[0] == "actuation"][0]
        out["actions"].append(actions)
        out["phys_dof"].append(dof)
        out["noise"].append(noise)
        out["reset_mask"].append(mask)
        out["obs"].append(obs_dict["obs"].clone())
        out["rew"].append(rew.clone())
        out["reset"].append(reset.clone())
        out["progress"].append(env.progress_buf.clone())
        out["timeouts"].append(extras["time_outs"].clone().long())
        out["dof_after"].append(env.dof_state.view(N, 2, 2).clone())
        out["reset_in"].append(reset_in)
        out["progress_in"].append(progress_in)
        out["actuation"].append(act.view(N, 2).clone())
    return {k: torch.stack(v) for k, v in out.items()}


class FakeHandGym(FakeGym):
    """FakeGym + the asset/actor surface of tasks/shadow_hand.py:220-396 (3 actors per env)."""

    def __init__(self, spec, num_envs, gen):
        super().__init__(spec, num_envs)
        self.nb = spec["nbodies"] + 2
        self.rbs = torch.zeros(num_envs * self.nb, 13)
        self.targets = None
        self.gen = gen
        self.env = None
        self.record = None
        self._envs = 0

    def get_asset_rigid_shape_count(self, a):
        return 22

    def load_asset(self, sim, root, path, *a):
        return path

    def get_asset_rigid_body_count(self, a):
        # the hand MJCF has the articulation's bodies; the object and goal URDFs one body each
        return len(self.spec["bodies"]) if "shadow_hand" in str(a) else 1

    def get_asset_actuator_count(self, a):
        return len(self.spec["actuated"])

    def get_asset_tendon_count(self, a):
        return len(self.spec["tendons"])

    def get_asset_tendon_properties(self, a):
        return [_Prop(limit_stiffness=0.0, damping=0.0) for _ in self.spec["tendons"]]

    def get_asset_tendon_name(self, a, i):
        return self.spec["tendons"][i]

    def set_asset_tendon_properties(self, a, props):
        self.tendon_props = props

    def get_asset_actuator_joint_name(self, a, i):
        return self.spec["dof_names"][self.spec["actuated"][i]]

    def find_asset_dof_index(self, a, name):
        return self.spec["dof_names"].index(name)

    def get_asset_dof_properties(self, a):
        return {"lower": np.array(self.spec["lower"], np.float32), "upper": np.array(self.spec["upper"], np.float32)}

    def create_env(self, *a):
        self._envs += 1
        return self._envs - 1

    def begin_aggregate(self, *a):
        pass

    end_aggregate = begin_aggregate

    def create_actor(self, env, asset, pose, name, group, filt, seg):
        return {"hand": 0, "object": 1, "goal_object": 2}[name]

    def get_actor_index(self, env, handle, domain):
        return 3 * env + handle

    def get_actor_rigid_body_properties(self, env, h):
        return [_Prop(mass=0.070875)]

    def get_sim_dof_count(self, sim):
        return self.N * self.spec["num_dof"]

    def acquire_rigid_body_state_tensor(self, sim):
        return self.rbs

    refresh_rigid_body_state_tensor = FakeGym.refresh_dof_state_tensor

    def set_dof_state_tensor_indexed(self, sim, data, idx, n):
        # hand actors carry global actor indices 3 * env (shadow_hand.py:657-663)
        nd = self.spec["num_dof"]
        e = idx.long() // 3
        self.dof.view(self.N, nd, 2)[e] = data.view(self.N, nd, 2)[e]
        self.calls.append(("dof_indexed", idx.clone()))

    def set_dof_position_target_tensor_indexed(self, sim, data, idx, n):
        self.calls.append(("target_indexed", idx.clone()))

    def set_dof_position_target_tensor(self, sim, t):
        self.targets = t.clone()

    def apply_rigid_body_force_tensors(self, sim, forces, torques, space):
        self.calls.append(("rb_forces", forces.clone(), int(space)))

    def simulate(self, sim):
        N, nd, g = self.N, self.spec["num_dof"], self.gen
        rec = {"root_pre": self.root.view(N, 3, 13).clone(), "dof_pre": self.dof.view(N, nd, 2).clone(),
               "targets": self.targets.clone()}
        root = self.root.view(N, 3, 13).clone()
        goal = self.env.goal_states
        obj = root[:, 1]
        obj[:, 0:3] = goal[:, 0:3] + torch.randn(N, 3, generator=g) * 0.12
        q = torch.randn(N, 4, generator=g)
        q = q / q.norm(dim=-1, keepdim=True)
        near = torch.rand(N, generator=g) < 0.3          # some envs reach the goal orientation (success)
        q[near] = goal[near, 3:7]
        obj[:, 3:7] = q
        obj[:, 7:13] = torch.randn(N, 6, generator=g)
        lo = torch.tensor(self.spec["lower"])
        hi = torch.tensor(self.spec["upper"])
        pos = lo + (hi - lo) * (torch.rand(N, nd, generator=g) * 1.1 - 0.05)
        dof = torch.stack([pos, torch.randn(N, nd, generator=g) * 2], -1)
        rbs = torch.randn(N, self.nb, 13, generator=g)
        sens = torch.randn(N * 5, 6, generator=g)
        dforce = torch.randn(N * nd, generator=g)
        self.root.copy_(root.view(N * 3, 13))
        self.dof.copy_(dof.view(N * nd, 2))
        self.rbs.copy_(rbs.view(-1, 13))
        self.sensors.copy_(sens)
        self.dof_force.copy_(dforce)
        rec.update(phys_root=root.clone(), phys_dof=dof.clone(), phys_rbs=rbs.clone(), phys_sensors=sens.view(N, 30),
                   phys_dof_force=dforce.view(N, nd))
        self.record = rec


class _TorchRecorder:
    """Stands in for a task module's ``torch``: every ``torch.rand`` / ``torch.randn`` draw is kept."""

    def __init__(self):
        self.draws = []

    def __getattr__(self, k):
        return getattr(torch, k)

    def rand(self, *shape, **kw):
        u = torch.rand(*shape, **kw)
        self.draws.append(("rand", u.clone()))
        return u

    def randn(self, *shape, **kw):
        u = torch.randn(*shape, **kw)
        self.draws.append(("randn", u.clone()))
        return u


def run_shadowhand(N=32, T=8, ep_len=4, obs_type="full_state", force_scale=0.0, asymmetric=False,
                   force_prob_range=None, object_type="block"):
    import importlib
    sys.path.insert(0, os.path.join(HERE, "..", "..", "isaacgymenvs-ma_amd"))
    from migym import model as M
    mod = importlib.import_module("isaacgymenvs.tasks.shadow_hand")
    hand = M.load_builtin("shadow_hand")
    actuated = [hand.dof_index(a["joint"]) for a in hand.actuators]
    spec = dict(num_dof=hand.num_dofs, sensors=5, actors=3, nbodies=len(hand.bodies),
                bodies=[b.name for b in hand.bodies], dof_names=hand.dof_names, actuated=actuated,
                tendons=["robot0:T_FFJ1c", "robot0:T_MFJ1c", "robot0:T_RFJ1c", "robot0:T_LFJ1c"],
                lower=[n.lower for n in hand.nodes[1:]], upper=[n.upper for n in hand.nodes[1:]], gears=[])
    fake = FakeHandGym(spec, N, torch.Generator().manual_seed(3))
    install_fake(fake)
    rec = RandRecorder()
    mod.torch_rand_float = rec
    trec = _TorchRecorder()
    mod.torch = trec
    cfg = load_task_cfg("ShadowHand", N, ep_len)
    cfg["env"]["observationType"] = obs_type
    cfg["env"]["forceScale"] = force_scale
    cfg["env"]["asymmetric_observations"] = asymmetric
    cfg["env"]["objectType"] = object_type
    if force_prob_range is not None:
        cfg["env"]["forceProbRange"] = force_prob_range
    torch.manual_seed(0)
    env = mod.ShadowHand(cfg, "cpu", "cpu", -1, True, False, False)
    init_force_prob = env.random_force_prob.clone()
    fake.env = env
    nd = spec["num_dof"]
    g = torch.Generator().manual_seed(4)
    keys = ("actions", "noise", "reset_in", "reset_goal_in", "progress_in", "root_pre", "dof_pre", "targets",
            "prev_targets", "goal_states", "phys_root", "phys_dof", "phys_rbs", "phys_sensors", "phys_dof_force",
            "obs", "rew", "reset", "reset_goal", "progress", "successes", "cons", "timeouts", "rb_forces",
            "force_prob", "states")
    out = {k: [] for k in keys}
    out["init_root"] = env.root_state_tensor.view(N, 3, 13).clone()
    out["init_goal_states"] = env.goal_states.clone()
    for t in range(T):
        actions = torch.rand(N, env.num_actions, generator=g) * 2.4 - 1.2
        reset_in, goal_in = env.reset_buf.clone(), env.reset_goal_buf.clone()
        progress_in = env.progress_buf.clone()
        rec.draws.clear()
        trec.draws.clear()
        obs_dict, rew, reset, extras = env.step(actions)
        noise = torch.zeros(N, 66)
        gids = goal_in.nonzero(as_tuple=False).flatten()
        eids = reset_in.nonzero(as_tuple=False).flatten()
        k = 0
        if len(gids) > 0:
            noise[gids, 0:4] = rec.draws[0]
            k = 1
        if len(eids) > 0:
            noise[eids, 4:57] = rec.draws[k]
            noise[eids, 57:61] = rec.draws[k + 1]
        # torch.rand / randn draws of the module, in call order: reset_idx's force-probability redraw
        # (shadow_hand.py:642-643), then with forceScale > 0 the selection U(0,1) over all envs and the
        # N(0,1) force rows of the selected envs (704-706)
        td = list(trec.draws)
        if len(eids) > 0:
            kind, u = td.pop(0)
            assert kind == "rand" and u.shape == (len(eids),)
            noise[eids, 61] = u
        if force_scale > 0.0:
            kind, u = td.pop(0)
            assert kind == "rand" and u.shape == (N,)
            noise[:, 62] = u
            sel = (u < env.random_force_prob).nonzero(as_tuple=False).flatten()
            kind, gn = td.pop(0)
            assert kind == "randn" and gn.shape[0] == len(sel)
            noise[sel, 63:66] = gn.reshape(len(sel), 3)
        assert not td, [d[0] for d in td]
        r = fake.record
        out["actions"].append(actions)
        out["noise"].append(noise)
        out["reset_in"].append(reset_in)
        out["reset_goal_in"].append(goal_in)
        out["progress_in"].append(progress_in)
        for kk in ("root_pre", "dof_pre", "targets", "phys_root", "phys_dof", "phys_rbs", "phys_sensors",
                   "phys_dof_force"):
            out[kk].append(r[kk])
        out["prev_targets"].append(env.prev_targets.clone())
        out["goal_states"].append(env.goal_states.clone())
        out["obs"].append(obs_dict["obs"].clone())
        out["rew"].append(rew.clone())
        out["reset"].append(reset.clone())
        out["reset_goal"].append(env.reset_goal_buf.clone())
        out["progress"].append(env.progress_buf.clone())
        out["successes"].append(env.successes.clone())
        out["cons"].append(env.consecutive_successes.clone())
        out["timeouts"].append(extras["time_outs"].clone().long())
        out["rb_forces"].append(env.rb_forces.clone())
        out["force_prob"].append(env.random_force_prob.clone())
        out["states"].append(obs_dict["states"].clone() if asymmetric else torch.zeros(N, 0))
    res = {k: (torch.stack(v) if isinstance(v, list) else v) for k, v in out.items()}
    res["episode_length"] = torch.tensor(ep_len)
    res["obs_type"] = np.array(obs_type)
    res["init_force_prob"] = init_force_prob
    res["force_scale"] = torch.tensor(force_scale)
    res["object_mass"] = torch.tensor(0.070875)
    res["object_type"] = np.array(object_type)
    return res


# ---------------------------------------------------------------------------------- domain randomization
DR_TRACE_PARAMS = {
    "frequency": 3,
    "observations": {"range": [0, .002], "range_correlated": [0, .001], "operation": "additive",
                     "distribution": "gaussian"},
    "actions": {"range": [0., .05], "range_correlated": [0, .015], "operation": "additive", "distribution": "uniform"},
    "sim_params": {"gravity": {"range": [0, 0.4], "operation": "additive", "distribution": "gaussian",
                               "schedule": "linear", "schedule_steps": 6}},
    "actor_params": {"ant": {
        "color": True,
        "rigid_body_properties": {"mass": {"range": [0.5, 1.5], "operation": "scaling", "distribution": "uniform",
                                           "setup_only": True}},
        "rigid_shape_properties": {"friction": {"num_buckets": 40, "range": [0.7, 1.3], "operation": "scaling",
                                                "distribution": "uniform", "schedule": "linear", "schedule_steps": 6},
                                   "restitution": {"range": [0., 0.7], "operation": "scaling",
                                                   "distribution": "uniform"}},
        "dof_properties": {"damping": {"range": [0.5, 1.5], "operation": "scaling", "distribution": "uniform",
                                       "schedule": "linear", "schedule_steps": 6},
                           "stiffness": {"range": [0.5, 1.5], "operation": "scaling", "distribution": "loguniform"},
                           "lower": {"range": [0, 0.01], "operation": "additive", "distribution": "gaussian"},
                           "upper": {"range": [0, 0.01], "operation": "additive", "distribution": "gaussian"}}}},
}


class _NpRandomRecorder:
    """Stands in for dr_utils' ``np``: np.random.normal / uniform draws are kept in call order."""

    def __init__(self):
        self.draws = []
        rec = self

        class _R:
            def normal(self, *a, **k):
                x = np.random.normal(*a, **k)
                rec.draws.append(np.array(x, dtype=np.float64).ravel())
                return x

            def uniform(self, *a, **k):
                x = np.random.uniform(*a, **k)
                rec.draws.append(np.array(x, dtype=np.float64).ravel())
                return x
        self.random = _R()

    def __getattr__(self, k):
        return getattr(np, k)


class FakeDRGym(FakeGym):
    """FakeGym + the property getters/setters apply_randomizations uses (vec_task.py:612-842)."""

    def __init__(self, spec, num_envs, hand):
        super().__init__(spec, num_envs)
        from isaacgym import gymapi as ga
        self.model = hand
        self.frames = 0
        self.simp = ga.SimParams()
        self.simp.gravity = ga.Vec3(0.0, 0.0, -9.81)
        self.simp.physx.rest_offset = 0.0
        self.sim_param_sets = []
        n, nd = num_envs, spec["num_dof"]
        self.dof_set = {k: np.zeros((n, nd)) for k in ("damping", "stiffness", "lower", "upper")}
        self.mass_set = np.zeros((n, len(hand.bodies)))
        self.fric_set = np.zeros((n, len(hand.geoms)))
        self._envs = 0

    def create_env(self, *a):
        self._envs += 1
        return self._envs - 1

    def get_frame_count(self, sim):
        return self.frames

    def simulate(self, sim):
        super().simulate(sim)
        self.frames += 1

    def get_sim_params(self, sim):
        # gym.get_sim_params returns the parameters by value (a new pybind object per call)
        from isaacgym import gymapi as ga
        q = ga.SimParams()
        q.gravity = ga.Vec3(self.simp.gravity.x, self.simp.gravity.y, self.simp.gravity.z)
        q.physx.rest_offset = self.simp.physx.rest_offset
        return q

    def set_sim_params(self, sim, p):
        self.simp.gravity.x, self.simp.gravity.y, self.simp.gravity.z = p.gravity.x, p.gravity.y, p.gravity.z
        self.sim_param_sets.append((p.gravity.x, p.gravity.y, p.gravity.z))

    def find_actor_handle(self, env, name):
        return 0

    def get_actor_count(self, env):
        return 1

    def get_actor_handle(self, env, i):
        return 0

    def get_actor_name(self, env, h):
        return "ant"

    def get_actor_rigid_shape_count(self, env, h):
        return len(self.model.geoms)

    def get_actor_rigid_body_count(self, env, h):
        return len(self.model.bodies)

    def get_actor_dof_properties(self, env, h):
        nd = self.spec["num_dof"]
        dt = np.dtype([("hasLimits", "?"), ("lower", "f4"), ("upper", "f4"), ("driveMode", "i4"), ("velocity", "f4"),
                       ("effort", "f4"), ("stiffness", "f4"), ("damping", "f4"), ("friction", "f4"),
                       ("armature", "f4")])
        a = np.zeros(nd, dt)
        nodes = self.model.nodes[1:]
        a["hasLimits"] = True
        a["lower"] = [x.lower for x in nodes]
        a["upper"] = [x.upper for x in nodes]
        a["stiffness"] = [x.stiffness for x in nodes]
        a["damping"] = [x.damping for x in nodes]
        a["armature"] = [x.armature for x in nodes]
        return a

    def set_actor_dof_properties(self, env, h, props):
        if isinstance(env, int):
            for k in self.dof_set:
                self.dof_set[k][env] = props[k]

    def get_actor_rigid_body_properties(self, env, h):
        return [_Prop(mass=float(self.model.nodes[b.node].mass)) for b in self.model.bodies]

    def set_actor_rigid_body_properties(self, env, h, props, recompute=False):
        self.mass_set[env] = [float(np.asarray(p.mass).ravel()[0]) for p in props]

    def get_actor_rigid_shape_properties(self, env, h):
        return [_Prop(friction=1.0, restitution=0.0) for _ in self.model.geoms]

    def set_actor_rigid_shape_properties(self, env, h, props):
        self.fric_set[env] = [float(np.asarray(p.friction).ravel()[0]) for p in props]

    def get_actor_tendon_properties(self, env, h):
        return []

    def set_actor_tendon_properties(self, env, h, props):
        pass


def run_ant_dr(N=32, T=10, ep_len=3):
    """Ant with task.randomize on the fake gym: every numpy / torch draw of apply_randomizations and of the
    noise lambdas is recorded, with the property values the reference hands to the gym setters."""
    import importlib
    sys.path.insert(0, os.path.join(HERE, "..", "..", "isaacgymenvs-ma_amd"))
    from migym import model as M
    from isaacgymenvs.utils import dr_utils
    import isaacgymenvs.tasks.base.vec_task as vt
    mod = importlib.import_module("isaacgymenvs.tasks.ant")
    ant = M.load_builtin("ant")
    d = math.pi / 180
    spec = dict(num_dof=8, sensors=4, start_z=0.44, gears=[15.0] * 8, bodies=[b.name for b in ant.bodies],
                lower=[x * d for x in [-40, 30, -40, -100, -40, -100, -40, 30]],
                upper=[x * d for x in [40, 100, 40, -30, 40, -30, 40, 100]])
    fake = FakeDRGym(spec, N, ant)
    install_fake(fake)
    rec = RandRecorder()
    mod.torch_rand_float = rec
    nprec = _NpRandomRecorder()
    dr_utils.np = nprec
    trec = _TorchRecorder()

    def randn_like(t, *a, **k):
        u = torch.randn_like(t, *a, **k)
        trec.draws.append(("randn", u.clone()))
        return u

    def rand_like(t, *a, **k):
        u = torch.rand_like(t, *a, **k)
        trec.draws.append(("rand", u.clone()))
        return u
    trec.randn_like, trec.rand_like = randn_like, rand_like
    vt.torch = trec
    cfg = load_task_cfg("Ant", N, ep_len)
    cfg["task"]["randomize"] = True
    cfg["task"]["randomization_params"] = DR_TRACE_PARAMS
    np.random.seed(7)
    torch.manual_seed(0)
    env = mod.Ant(cfg, "cpu", "cpu", -1, True, False, False)
    out = {"init_np": [np.concatenate(nprec.draws)], "init_sim": [fake.sim_param_sets[-1]],
           "init_mass": [fake.mass_set.copy()], "init_fric": [fake.fric_set.copy()],
           "init_dof": [np.stack([fake.dof_set[k].copy() for k in ("damping", "stiffness", "lower", "upper")])]}
    nprec.draws.clear()
    keys = ("actions", "act_draws", "obs_draws", "np_draws", "sim_set", "actuation", "phys_root", "phys_dof",
            "phys_sensors", "noise", "reset_in", "progress_in", "obs", "rew", "reset", "progress", "randomize_buf",
            "mass_set", "fric_set", "dof_set", "potentials", "prev_potentials")
    for k in keys:
        out[k] = []
    nd = 8
    lo, hi = torch.tensor(spec["lower"]), torch.tensor(spec["upper"])
    lo, hi = torch.minimum(lo, hi), torch.maximum(lo, hi)
    g = torch.Generator().manual_seed(5)
    for t in range(T):
        actions = torch.rand(N, 8, generator=g) * 2.4 - 1.2
        root, dof, sens = physics_output(g, N, nd, lo, hi, (0.25, 0.7), 4)
        fake.inject = (root, dof, sens, None)
        reset_in, progress_in = env.reset_buf.clone(), env.progress_buf.clone()
        rec.draws.clear()
        trec.draws.clear()
        nprec.draws.clear()
        fake.calls.clear()
        nsim = len(fake.sim_param_sets)
        obs_dict, rew, reset, extras = env.step(actions)
        ids = reset_in.nonzero(as_tuple=False).flatten()
        noise = torch.zeros(N, 2 * nd)
        if len(ids) > 0:
            noise[ids, :nd] = rec.draws[0]
            noise[ids, nd:] = rec.draws[1]
        # torch draws: the action lambda's (N, 8) [corr?, z] then the observation lambda's (N, 60) [corr?, z]
        act = [u for _, u in trec.draws if u.shape[-1] == 8]
        obsd = [u for _, u in trec.draws if u.shape[-1] == 60]
        pad = lambda lst, w: torch.stack(lst + [torch.full((N, w), float("nan"))] * (2 - len(lst)))  # noqa: E731
        out["act_draws"].append(pad(act, 8) if len(act) == 2 else torch.stack([torch.full((N, 8), float("nan")), act[0]]))
        out["obs_draws"].append(pad(obsd, 60) if len(obsd) == 2 else torch.stack([torch.full((N, 60), float("nan")), obsd[0]]))
        nd_np = np.concatenate(nprec.draws) if nprec.draws else np.zeros(0)
        out["np_draws"].append(nd_np)
        out["sim_set"].append(np.array(fake.sim_param_sets[nsim:] or [(np.nan,) * 3]))
        out["actions"].append(actions)
        out["actuation"].append([c[1] for c in fake.calls if c[0] == "actuation"][0].view(N, nd).clone())
        out["phys_root"].append(root)
        out["phys_dof"].append(dof.view(N, nd, 2))
        out["phys_sensors"].append(sens.view(N, 24))
        out["noise"].append(noise)
        out["reset_in"].append(reset_in)
        out["progress_in"].append(progress_in)
        out["obs"].append(obs_dict["obs"].clone())
        out["rew"].append(rew.clone())
        out["reset"].append(reset.clone())
        out["progress"].append(env.progress_buf.clone())
        out["randomize_buf"].append(env.randomize_buf.clone())
        out["mass_set"].append(fake.mass_set.copy())
        out["fric_set"].append(fake.fric_set.copy())
        out["dof_set"].append(np.stack([fake.dof_set[k].copy() for k in ("damping", "stiffness", "lower", "upper")]))
        out["potentials"].append(env.potentials.clone())
        out["prev_potentials"].append(env.prev_potentials.clone())
    res = {}
    for k, v in out.items():
        if k in ("np_draws", "sim_set", "init_np"):
            # ragged: concatenate with per-step lengths
            res[k + "_len"] = np.array([len(x) for x in v])
            res[k] = np.concatenate([np.asarray(x, np.float64).reshape(len(x), -1) if k == "sim_set"
                                     else np.asarray(x, np.float64).reshape(-1, 1) for x in v])
        else:
            res[k] = torch.stack(v) if isinstance(v[0], torch.Tensor) else np.stack(v)
    res["episode_length"] = torch.tensor(ep_len)
    res["lower"], res["upper"] = lo, hi
    return res


def save(name, d):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: (v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v))
                                 for k, v in d.items()})
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    # one task per process: vec_task keeps a process-global sim (vec_task.py:55-64)
    if which == "all":
        import subprocess
        for t in ("ant", "humanoid", "cartpole", "shadowhand", "shadowhand_obs", "shadowhand_forces", "shadowhand_pen", "ant_dr",
                  "ant_reset_done", "humanoid_reset_done"):
            subprocess.check_call([sys.executable, __file__, t])
        return
    if which == "ant":
        save("trace_ant.npz", run_locomotion("Ant"))
    elif which == "humanoid":
        save("trace_humanoid.npz", run_locomotion("Humanoid"))
    elif which in ("ant_reset_done", "humanoid_reset_done"):  # step -> reset_done -> step (vec_task.py:442-457)
        task = "Ant" if which.startswith("ant") else "Humanoid"
        save(f"trace_{task.lower()}_reset_done.npz", run_locomotion(task, N=64, T=7, ep_len=4, reset_done=True))
    elif which == "cartpole":
        save("trace_cartpole.npz", run_cartpole())
    elif which == "shadowhand":
        save("trace_shadowhand.npz", run_shadowhand())
    elif which == "ant_dr":  # task.randomize: property draws, noise lambdas, gravity
        save("trace_ant_dr.npz", run_ant_dr())
    elif which == "shadowhand_forces":  # random object forces + asymmetric states (forceScale > 0)
        save("trace_shadowhand_forces.npz", run_shadowhand(N=32, T=8, ep_len=4, force_scale=2.0, asymmetric=True,
                                                               force_prob_range=[0.2, 0.8]))
    elif which == "shadowhand_pen":  # objectType pen: randomize_rotation_pen resets, ignore_z_rot reward
        save("trace_shadowhand_pen.npz", run_shadowhand(N=32, T=8, ep_len=4, object_type="pen"))
    elif which == "shadowhand_obs":  # the other observationType layouts, smaller traces
        for ot in ("full", "full_no_vel", "openai"):
            save(f"trace_shadowhand_{ot}.npz", run_shadowhand(N=16, T=4, ep_len=3, obs_type=ot))


if __name__ == "__main__":
    main()
