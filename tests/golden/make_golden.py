#!/usr/bin/env python3
"""Generate golden input/output vectors from the reference's own jit functions.

Run in the build container only (needs /root/reference):

    python tests/golden/make_golden.py

Writes ``tests/golden/jit_*.npz``.  Each file holds seeded, physically plausible
inputs plus the outputs the REFERENCE functions produced for them, including
adversarial rows (yaw wrap, thresholds, |quat_diff| clamp).  These pin the
oracle (oracle/) and, through it, the HIP kernels.  Functions exercised
(file:line in the reference):

  utils/torch_jit_utils.py:41-62   quat_mul        :65-67  normalize
  utils/torch_jit_utils.py:70-77   quat_apply      :80-103 quat_rotate[_inverse]
  utils/torch_jit_utils.py:106-110 quat_conjugate  :118-123 quat_from_angle_axis
  utils/torch_jit_utils.py:126-128 normalize_angle :175-195 get_euler_xyz
  utils/torch_jit_utils.py:228-240 tensor_clamp / scale / unscale
  utils/torch_jit_utils.py:247-276 compute_heading_and_up / compute_rot
  tasks/ant.py:325-408             compute_ant_reward / compute_ant_observations
  tasks/humanoid.py:323-413        compute_humanoid_reward / _observations
  tasks/cartpole.py:180-196        compute_cartpole_reward
  tasks/shadow_hand.py:746-806     compute_hand_reward / randomize_rotation
"""
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refshim  # noqa: E402

_refshim.install()
from isaacgymenvs.utils import torch_jit_utils as tju  # noqa: E402

N = 256


def unit_quats(g, n):
    q = torch.randn(n, 4, generator=g)
    q = q / q.norm(dim=-1, keepdim=True)
    return q


def yawish_quats(g, n):
    """Mostly-upright torsos: small roll/pitch, any yaw (exercises yaw wrap)."""
    yaw = (torch.rand(n, generator=g) * 2 - 1) * math.pi
    roll = (torch.rand(n, generator=g) * 2 - 1) * 0.4
    pitch = (torch.rand(n, generator=g) * 2 - 1) * 0.4
    return tju.quat_from_euler_xyz(roll, pitch, yaw)


def adversarial_quats():
    s = math.sqrt(0.5)
    return torch.tensor([
        [0, 0, 0, 1.0],            # identity: yaw exactly 0
        [0, 0, 1e-7, 1.0],         # yaw just above 0
        [0, 0, -1e-7, 1.0],        # yaw just below 0 -> wraps to ~2pi
        [0, 0, 1.0, 0.0],          # yaw = pi
        [0, 0, s, s],              # yaw = pi/2
        [0, 0, -s, s],             # yaw = -pi/2 -> 3pi/2
        [s, 0, 0, s],              # roll = pi/2
        [0, s, 0, s],              # pitch = pi/2 (asin clamp path)
        [0, -s, 0, s],             # pitch = -pi/2
        [1.0, 0, 0, 0],            # upside down
    ], dtype=torch.float32)


def with_adv(q):
    a = adversarial_quats()
    a = a / a.norm(dim=-1, keepdim=True)
    q = q.clone()
    q[: a.shape[0]] = a
    return q


def gen_tju(g):
    a = unit_quats(g, N)
    b = unit_quats(g, N)
    v = torch.randn(N, 3, generator=g) * 3
    x = torch.randn(N, 3, generator=g)
    x[0] = 0.0  # normalize eps clamp path
    ang = (torch.rand(N, generator=g) * 2 - 1) * 10.0
    ang[:4] = torch.tensor([math.pi, -math.pi, 3 * math.pi, 0.0])
    axis = torch.randn(N, 3, generator=g)
    qe = with_adv(unit_quats(g, N))
    lo = -torch.rand(N, 5, generator=g) - 0.1
    hi = torch.rand(N, 5, generator=g) + 0.1
    t = torch.randn(N, 5, generator=g)
    rot = with_adv(yawish_quats(g, N))
    inv_start = tju.quat_conjugate(unit_quats(g, 1)).repeat(N, 1)
    to_target = torch.randn(N, 3, generator=g) * 100
    to_target[:, 2] = 0
    vec0 = torch.tensor([[1.0, 0, 0]]).repeat(N, 1)
    vec1 = torch.tensor([[0, 0, 1.0]]).repeat(N, 1)
    targets = torch.tensor([[1000.0, 0, 0]]).repeat(N, 1)
    pos = torch.randn(N, 3, generator=g)
    vel = torch.randn(N, 3, generator=g)
    avel = torch.randn(N, 3, generator=g)
    out = {}
    out["a"], out["b"], out["v"], out["x"] = a, b, v, x
    out["ang"], out["axis"], out["qe"] = ang, axis, qe
    out["lo"], out["hi"], out["t"] = lo, hi, t
    out["rot"], out["inv_start"], out["to_target"] = rot, inv_start, to_target
    out["vec0"], out["vec1"], out["targets"], out["pos"] = vec0, vec1, targets, pos
    out["vel"], out["avel"] = vel, avel
    out["quat_mul"] = tju.quat_mul(a, b)
    out["quat_conjugate"] = tju.quat_conjugate(a)
    out["quat_apply"] = tju.quat_apply(a, v)
    out["quat_rotate"] = tju.quat_rotate(a, v)
    out["quat_rotate_inverse"] = tju.quat_rotate_inverse(a, v)
    out["normalize"] = tju.normalize(x)
    out["normalize_angle"] = tju.normalize_angle(ang)
    out["quat_from_angle_axis"] = tju.quat_from_angle_axis(ang, axis)
    r, p, y = tju.get_euler_xyz(qe)
    out["euler_roll"], out["euler_pitch"], out["euler_yaw"] = r, p, y
    out["scale"] = tju.scale(t, lo, hi)
    out["unscale"] = tju.unscale(t, lo, hi)
    out["tensor_clamp"] = tju.tensor_clamp(t, lo, hi)
    tq, up_proj, head_proj, up_vec, head_vec = tju.compute_heading_and_up(rot, inv_start, to_target, vec0, vec1, 2)
    out["hu_torso_quat"], out["hu_up_proj"], out["hu_heading_proj"] = tq, up_proj, head_proj
    out["hu_up_vec"], out["hu_heading_vec"] = up_vec, head_vec
    vl, al, rr, pp, yy, att = tju.compute_rot(tq, vel, avel, targets, pos)
    out["rot_vel_loc"], out["rot_angvel_loc"], out["rot_roll"] = vl, al, rr
    out["rot_pitch"], out["rot_yaw"], out["rot_angle_to_target"] = pp, yy, att
    return out


def ant_limits():
    d = math.pi / 180.0
    lo = torch.tensor([-40, 30, -40, -100, -40, -100, -40, 30], dtype=torch.float32) * d
    hi = torch.tensor([40, 100, 40, -30, 40, -30, 40, 100], dtype=torch.float32) * d
    return lo, hi


def humanoid_limits():
    deg = [(-45, 45), (-75, 30), (-35, 35), (-45, 15), (-60, 35), (-120, 45), (-160, 2), (-50, 50), (-50, 50),
           (-45, 15), (-60, 35), (-120, 45), (-160, 2), (-50, 50), (-50, 50), (-90, 70), (-90, 70), (-90, 50),
           (-90, 70), (-90, 70), (-90, 50)]
    lo = torch.tensor([a for a, _ in deg], dtype=torch.float32) * math.pi / 180
    hi = torch.tensor([b for _, b in deg], dtype=torch.float32) * math.pi / 180
    return lo, hi


def locomotion_state(g, nd, z_lo, z_hi, lo, hi, nsens):
    root = torch.zeros(N, 13)
    root[:, 0:2] = (torch.rand(N, 2, generator=g) * 2 - 1) * 5
    root[:, 2] = z_lo + (z_hi - z_lo) * torch.rand(N, generator=g)
    root[:, 3:7] = with_adv(yawish_quats(g, N))
    root[:, 7:13] = torch.randn(N, 6, generator=g)
    u = torch.rand(N, nd, generator=g)
    dof_pos = lo + u * (hi - lo)
    dof_pos[1] = hi  # exactly at upper limit -> unscale == 1 (> 0.99 cost path)
    dof_pos[2] = lo
    dof_vel = torch.randn(N, nd, generator=g) * 2
    sensors = torch.randn(N, nsens, generator=g) * 20
    actions = torch.rand(N, nd, generator=g) * 2 - 1
    potentials = -1000.0 / 0.0166 + torch.randn(N, generator=g)
    return root, dof_pos, dof_vel, sensors, actions, potentials


def gen_ant(g):
    from isaacgymenvs.tasks import ant as ant_mod
    lo, hi = ant_limits()
    root, dof_pos, dof_vel, sensors, actions, potentials = locomotion_state(g, 8, 0.2, 0.8, lo, hi, 24)
    root[3, 2] = 0.31  # exactly at termination height
    targets = torch.tensor([[1000.0, 0, 0]]).repeat(N, 1)
    inv_start = tju.quat_conjugate(torch.tensor([[0, 0, 0, 1.0]])).repeat(N, 1)
    b0 = torch.tensor([[1.0, 0, 0]]).repeat(N, 1)
    b1 = torch.tensor([[0, 0, 1.0]]).repeat(N, 1)
    obs_in = torch.zeros(N, 60)
    obs, pot, prev_pot, up_vec, heading_vec = ant_mod.compute_ant_observations(
        obs_in, root, targets, potentials.clone(), inv_start, dof_pos, dof_vel, lo, hi, 0.2,
        sensors, actions, 0.0166, 0.1, b0, b1, 2)
    reset_buf = (torch.rand(N, generator=g) < 0.2).long()
    progress = torch.randint(0, 1000, (N,), generator=g)
    progress[:6] = torch.tensor([0, 997, 998, 999, 1000, 1])
    rew, reset = ant_mod.compute_ant_reward(obs, reset_buf, progress, actions, 0.1, 0.5, pot, prev_pot,
                                            0.005, 0.05, 0.1, 0.31, -2.0, 1000.0)
    return dict(root=root, dof_pos=dof_pos, dof_vel=dof_vel, sensors=sensors, actions=actions,
                potentials_in=potentials, targets=targets, inv_start=inv_start, lo=lo, hi=hi,
                obs=obs, potentials=pot, prev_potentials=prev_pot, up_vec=up_vec, heading_vec=heading_vec,
                reset_buf=reset_buf, progress=progress, rew=rew, reset=reset)


def gen_humanoid(g):
    from isaacgymenvs.tasks import humanoid as hum_mod
    lo, hi = humanoid_limits()
    root, dof_pos, dof_vel, sensors, actions, potentials = locomotion_state(g, 21, 0.6, 1.4, lo, hi, 12)
    root[3, 2] = 0.8
    dof_force = torch.randn(N, 21, generator=g) * 50
    targets = torch.tensor([[1000.0, 0, 0]]).repeat(N, 1)
    inv_start = torch.tensor([[0, 0, 0, 1.0]]).repeat(N, 1)
    b0 = torch.tensor([[1.0, 0, 0]]).repeat(N, 1)
    b1 = torch.tensor([[0, 0, 1.0]]).repeat(N, 1)
    obs_in = torch.zeros(N, 108)
    obs, pot, prev_pot, up_vec, heading_vec = hum_mod.compute_humanoid_observations(
        obs_in, root, targets, potentials.clone(), inv_start, dof_pos, dof_vel, dof_force, lo, hi, 0.1,
        sensors, actions, 0.0166, 0.01, 0.25, b0, b1)
    motor_efforts = torch.tensor([67.5, 67.5, 67.5, 45, 45, 135, 90, 22.5, 22.5, 45, 45, 135, 90, 22.5, 22.5,
                                  67.5, 67.5, 45, 67.5, 67.5, 45], dtype=torch.float32)
    reset_buf = (torch.rand(N, generator=g) < 0.2).long()
    progress = torch.randint(0, 1000, (N,), generator=g)
    progress[:6] = torch.tensor([0, 997, 998, 999, 1000, 1])
    rew, reset = hum_mod.compute_humanoid_reward(obs, reset_buf, progress, actions, 0.1, 0.5, pot, prev_pot,
                                                 0.01, 0.05, 0.25, 135.0, motor_efforts, 0.8, -1.0, 1000.0)
    return dict(root=root, dof_pos=dof_pos, dof_vel=dof_vel, dof_force=dof_force, sensors=sensors,
                actions=actions, potentials_in=potentials, targets=targets, inv_start=inv_start, lo=lo, hi=hi,
                obs=obs, potentials=pot, prev_potentials=prev_pot, up_vec=up_vec, heading_vec=heading_vec,
                motor_efforts=motor_efforts, reset_buf=reset_buf, progress=progress, rew=rew, reset=reset)


def gen_cartpole(g):
    from isaacgymenvs.tasks import cartpole as cp_mod
    dof = torch.randn(N, 4, generator=g) * torch.tensor([2.0, 1.0, 1.2, 2.0])
    dof[0, 0] = 3.0            # exactly at reset distance (not > )
    dof[1, 0] = 3.0001
    dof[2, 2] = math.pi / 2     # exactly at angle bound
    dof[3, 2] = -1.5708
    reset_buf = (torch.rand(N, generator=g) < 0.2).long()
    progress = torch.randint(0, 500, (N,), generator=g)
    progress[:5] = torch.tensor([0, 498, 499, 500, 497])
    rew, reset = cp_mod.compute_cartpole_reward(dof[:, 2], dof[:, 3], dof[:, 1], dof[:, 0], 3.0,
                                                reset_buf, progress, 500.0)
    return dict(obs=dof, reset_buf=reset_buf, progress=progress, rew=rew, reset=reset)


def gen_shadow(g):
    from isaacgymenvs.tasks import shadow_hand as sh_mod
    object_pos = torch.tensor([[0.0, -0.39, 0.6]]) + torch.randn(N, 3, generator=g) * 0.1
    target_pos = torch.tensor([[0.0, -0.39, 0.56]]).repeat(N, 1)
    object_pos[0] = target_pos[0] + torch.tensor([0.24, 0, 0])   # fall distance boundary
    object_rot = unit_quats(g, N)
    target_rot = unit_quats(g, N)
    target_rot[1] = object_rot[1]                                 # rot_dist == 0 (success)
    target_rot[2] = -object_rot[2]                                # q vs -q: |quat_diff xyz| clamp
    actions = torch.rand(N, 20, generator=g) * 2 - 1
    rew_buf = torch.zeros(N)
    reset_buf = (torch.rand(N, generator=g) < 0.1).long()
    reset_goal_buf = (torch.rand(N, generator=g) < 0.1).long()
    progress = torch.randint(0, 600, (N,), generator=g)
    progress[3:6] = torch.tensor([598, 599, 600])
    successes = torch.randint(0, 3, (N,), generator=g).float()
    cons = torch.tensor(0.7)
    outs = sh_mod.compute_hand_reward(rew_buf, reset_buf, reset_goal_buf, progress.clone(), successes, cons,
                                      600.0, object_pos, object_rot, target_pos, target_rot,
                                      -10.0, 1.0, 0.1, actions, -0.0002, 0.1, 250.0, 0.24, 0.0, 0, 0.1, False)
    r0 = torch.rand(N, generator=g) * 2 - 1
    r1 = torch.rand(N, generator=g) * 2 - 1
    xu = torch.tensor([[1.0, 0, 0]]).repeat(N, 1)
    yu = torch.tensor([[0, 1.0, 0]]).repeat(N, 1)
    rr = sh_mod.randomize_rotation(r0, r1, xu, yu)
    names = ["rew", "reset", "goal_reset", "progress_out", "successes_out", "cons_out"]
    d = dict(object_pos=object_pos, object_rot=object_rot, target_pos=target_pos, target_rot=target_rot,
             actions=actions, reset_buf=reset_buf, reset_goal_buf=reset_goal_buf, progress=progress,
             successes=successes, cons_in=cons, r0=r0, r1=r1, rand_rot=rr)
    d.update({k: v for k, v in zip(names, outs)})
    return d


def save(name, d):
    arrs = {}
    for k, v in d.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        arrs[k] = np.asarray(v)
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrs)
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def main():
    torch._C._jit_set_profiling_mode(False)
    torch._C._jit_set_profiling_executor(False)
    g = torch.Generator().manual_seed(0)
    save("jit_tju.npz", gen_tju(g))
    save("jit_ant.npz", gen_ant(g))
    save("jit_humanoid.npz", gen_humanoid(g))
    save("jit_cartpole.npz", gen_cartpole(g))
    save("jit_shadowhand.npz", gen_shadow(g))


if __name__ == "__main__":
    main()
