"""GPU test of the 8-GPU sharding on one card (BASELINE configs 4 and 5).

The multi-GPU configs run one process per GPU, each stepping the envs [rank * n, (rank + 1) * n) of the
node with `env_offset = rank * n` (migym/utils/rlgames_utils.py): every random draw (reset noise,
ShadowHand goal / object resets and random forces) is keyed by the global env / actor id, so a shard is
the corresponding slice of one big rollout.  Here the full node-size rollout and rank shards run on the
same GPU, with the same actions, and must agree bit for bit on obs, rew and reset at every step:

  * MA-Ant, 65,536 envs x 4 agents, shards of 8,192 envs (ranks 0, 3 and 7 of 8);
  * ShadowHand, 32,768 envs, shards of 4,096 (ranks 0 and 7 of 8);
  * Ant, 65,536 envs, shards of 8,192 (rank 5).

(The per-rank consecutive_successes mean is reduced across ranks by the dist layer and is not part of
obs / rew / reset.)  The tests that compare batches on both sides of the team-layout threshold (the
classic layout up to 2,048 waves, the compact one above; the two round differently) pin MIGYM_LAYOUT=compact, as a
deployment replaying a rank's shard alone would; the small-batch tests run the default choice.
"""
import os

import pytest
import torch

import migym
from migym import configs

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _make(task, n, offset):
    cfg = configs.task_config(task, n, sim_device=DEV)
    cfg["env_offset"] = offset
    return migym.make(seed=11, task=task, num_envs=n, sim_device=DEV, rl_device=DEV, headless=True,
                      cfg={"task": cfg})


@pytest.mark.parametrize("task,world,per_rank,ranks", [("MAAnt", 8, 8192, (0, 3, 7)),
                                                        ("ShadowHand", 8, 4096, (0, 7)),
                                                        ("Ant", 8, 8192, (5,))])
def test_rank_shards_equal_slices_of_the_node_rollout(task, world, per_rank, ranks, monkeypatch):
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    monkeypatch.setenv("MIGYM_LAYOUT", "compact")
    steps = 6
    full = _make(task, world * per_rank, 0)
    A = full.num_agents
    g = torch.Generator(device=DEV).manual_seed(5)
    acts = [torch.rand((full.num_actors, full.num_actions), device=DEV, generator=g) * 2.4 - 1.2 for _ in range(steps)]
    ref = []
    for a in acts:
        obs, rew, reset, _ = full.step(a)
        ref.append((obs["obs"].clone(), rew.clone(), reset.clone()))
    full.close()
    del full
    for r in ranks:
        sh = _make(task, per_rank, r * per_rank)
        lo, hi = r * per_rank * A, (r + 1) * per_rank * A
        for k, a in enumerate(acts):
            obs, rew, reset, _ = sh.step(a[lo:hi].contiguous())
            o, w, d = ref[k]
            assert torch.equal(obs["obs"], o[lo:hi]), f"{task} rank {r} step {k}: obs differ"
            assert torch.equal(rew, w[lo:hi]), f"{task} rank {r} step {k}: rew differ"
            assert torch.equal(reset, d[lo:hi]), f"{task} rank {r} step {k}: reset differ"
        assert int(d[lo:hi].sum()) >= 0
        sh.close()


@pytest.mark.parametrize("task,n,per_rank", [("Ant", 1 << 20, 8192), ("ShadowHand", 1 << 17, 4096)])
def test_largest_batch_equals_its_last_shard(task, n, per_rank, monkeypatch):
    """the large end of the size range: Ant at 1,048,576 envs (16x the headline, ~0.5 GB of state) and ShadowHand at
    131,072 envs (4x BASELINE configs[4]'s node total, one GPU), 4 steps; its last shard, stepped alone with
    env_offset = n - per_rank, must equal the batch's tail bit for bit (every index past 2^19 / 2^16 envs -- grid,
    work queue, counter RNG keys, row offsets -- as in the small runs)"""
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    monkeypatch.setenv("MIGYM_LAYOUT", "compact")
    steps = 4
    full = _make(task, n, 0)
    g = torch.Generator(device=DEV).manual_seed(9)
    acts = [torch.rand((full.num_actors, full.num_actions), device=DEV, generator=g) * 2.4 - 1.2 for _ in range(steps)]
    lo = n - per_rank
    ref = []
    for a in acts:
        obs, rew, reset, _ = full.step(a)
        assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
        ref.append((obs["obs"][lo:].clone(), rew[lo:].clone(), reset[lo:].clone()))
    full.close()
    del full
    torch.cuda.empty_cache()
    sh = _make(task, per_rank, lo)
    for k, a in enumerate(acts):
        obs, rew, reset, _ = sh.step(a[lo:].contiguous())
        o, w, d = ref[k]
        assert torch.equal(obs["obs"], o) and torch.equal(rew, w) and torch.equal(reset, d), f"{task} step {k}"
    sh.close()


@pytest.mark.parametrize("task,obj", [("Humanoid", "block"), ("ShadowHand", "egg"), ("ShadowHand", "pen")])
def test_work_queue_items_equal_the_static_grid(task, obj, monkeypatch):
    """Multi-wave-block instances (Humanoid: 4 waves per block, hand block / pen 2, egg 8) run a work queue
    (step_kernels.hpp wq_next): at 16,384 envs the waves dequeue most of their items from the device counter;
    a 2,048-env shard fits the resident grid and runs static items only.  Both must give the same envs the same
    bits, over consecutive launches (the counters are re-zeroed by the last wave of every launch)."""
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    monkeypatch.setenv("MIGYM_LAYOUT", "compact")
    steps, n, per = 4, 16384, 2048

    def make(num, offset):
        cfg = configs.task_config(task, num, sim_device=DEV)
        cfg["env_offset"] = offset
        if task == "ShadowHand":
            cfg["env"]["objectType"] = obj
        return migym.make(seed=3, task=task, num_envs=num, sim_device=DEV, rl_device=DEV, headless=True,
                          cfg={"task": cfg})

    full = make(n, 0)
    g = torch.Generator(device=DEV).manual_seed(9)
    acts = [torch.rand((full.num_actors, full.num_actions), device=DEV, generator=g) * 2.4 - 1.2 for _ in range(steps)]
    ref = []
    for a in acts:
        obs, rew, reset, _ = full.step(a)
        ref.append((obs["obs"].clone(), rew.clone(), reset.clone()))
    full.close()
    del full
    for r in (0, n // per - 1):
        sh = make(per, r * per)
        lo, hi = r * per, (r + 1) * per
        for k, a in enumerate(acts):
            obs, rew, reset, _ = sh.step(a[lo:hi].contiguous())
            o, w, d = ref[k]
            assert torch.equal(obs["obs"], o[lo:hi]), f"{task}/{obj} shard {r} step {k}: obs differ"
            assert torch.equal(rew, w[lo:hi]), f"{task}/{obj} shard {r} step {k}: rew differ"
            assert torch.equal(reset, d[lo:hi]), f"{task}/{obj} shard {r} step {k}: reset differ"
        sh.close()


@pytest.mark.parametrize("task,obj", [("Ant", "block"), ("Humanoid", "block"), ("MAAnt", "block"), ("Cartpole", "block"),
                                      ("ShadowHand", "block"), ("ShadowHand", "egg"), ("ShadowHand", "pen")])
def test_ragged_shards_equal_slices_of_one_rollout(task, obj):
    """Ragged env counts: shards of 1, 7, 67 and 225 envs at offsets 0, 1, 8 and 75 of one 300-env rollout (none a
    multiple of a wave's teams or of a block's waves, so every shard ends in a partly filled wave and the kernels'
    `slot < n` masks decide which lanes write).  Every shard must be the bit-identical slice of the full rollout
    over 6 steps with resets, and the full rollout must stay finite."""
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    steps, n = 6, 300
    cuts = [(0, 1), (1, 8), (8, 75), (75, 300)]

    def make(num, offset):
        cfg = configs.task_config(task, num, sim_device=DEV)
        cfg["env_offset"] = offset
        if task == "ShadowHand":
            cfg["env"]["objectType"] = obj
        return migym.make(seed=7, task=task, num_envs=num, sim_device=DEV, rl_device=DEV, headless=True,
                          cfg={"task": cfg})

    full = make(n, 0)
    A = full.num_agents
    g = torch.Generator(device=DEV).manual_seed(9)
    acts = [torch.rand((full.num_actors, full.num_actions), device=DEV, generator=g) * 2.4 - 1.2 for _ in range(steps)]
    ref = []
    for a in acts:
        obs, rew, reset, _ = full.step(a)
        ref.append((obs["obs"].clone(), rew.clone(), reset.clone()))
    full.close()
    del full
    assert all(torch.isfinite(o).all() for o, _, _ in ref)
    for lo_e, hi_e in cuts:
        sh = make(hi_e - lo_e, lo_e)
        lo, hi = lo_e * A, hi_e * A
        for k, a in enumerate(acts):
            obs, rew, reset, _ = sh.step(a[lo:hi].contiguous())
            o, w, d = ref[k]
            assert obs["obs"].shape[0] == hi - lo
            assert torch.equal(obs["obs"], o[lo:hi]), f"{task} envs [{lo_e}, {hi_e}) step {k}: obs differ"
            assert torch.equal(rew, w[lo:hi]), f"{task} envs [{lo_e}, {hi_e}) step {k}: rew differ"
            assert torch.equal(reset, d[lo:hi]), f"{task} envs [{lo_e}, {hi_e}) step {k}: reset differ"
        sh.close()


def _rollout_with_order(task, n, env_cfg, mode, steps):
    """`steps` fused steps of `task` with MIGYM_ORDER = mode (read at mg_sim_create), a short episode so that
    timeouts and terminations reset envs inside the run; every step's outputs and state, cloned"""
    old = os.environ.get("MIGYM_ORDER")
    os.environ["MIGYM_ORDER"] = mode
    try:
        cfg = configs.task_config(task, n, sim_device=DEV)
        cfg["env"].update(env_cfg)
        env = migym.make(seed=17, task=task, num_envs=n, sim_device=DEV, rl_device=DEV, headless=True,
                         cfg={"task": cfg})
    finally:
        if old is None:
            del os.environ["MIGYM_ORDER"]
        else:
            os.environ["MIGYM_ORDER"] = old
    g = torch.Generator(device=DEV).manual_seed(23)
    out = []
    for _ in range(steps):
        a = torch.rand((env.num_actors, env.num_actions), device=DEV, generator=g) * 2.4 - 1.2
        obs, rew, reset, extras = env.step(a)
        out.append((obs["obs"].clone(), rew.clone(), reset.clone(), env.root_states.clone(), env.dof_state.clone(),
                    env.progress_buf.clone()))
    resets = sum(int(o[2].sum()) for o in out[1:])
    env.close()
    return out, resets


@pytest.mark.parametrize("mode", ["lists", "sort"])
@pytest.mark.parametrize("task,n,env_cfg", [("Ant", 301, {}),
                                            ("Ant", 4099, {}),
                                            ("Humanoid", 301, {}),
                                            ("ShadowHand", 301, {"objectType": "block"}),
                                            ("ShadowHand", 301, {"objectType": "egg"}),
                                            ("ShadowHand", 301, {"objectType": "pen"}),
                                            ("MAAnt", 301, {"numAgents": 2})])
def test_work_order_changes_no_result(task, n, env_cfg, mode):
    """Work ordering (the in-kernel bucket lists, or the two-pass counting sort k_ohist / k_oscatter
    and its permutation) only changes which envs share a wave: ordering every step (MIGYM_ORDER=lists / sort, the
    first ordered launch the second step) and never (off) give the same obs, rew, reset, root and DOF state bit for
    bit over 12 steps with resets, on ragged env counts (the last wave and the sort's last block partly filled; Ant
    4,099: 17 sort blocks, so the blocks' global bin ranges interleave).  MAAnt with 2 agents per env is ordered by
    env units, so the agent alignment that the AND filter and the 'others' shuffles rely on is exercised under the
    permutation."""
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    env_cfg = dict(env_cfg, episodeLength=7)
    on, r_on = _rollout_with_order(task, n, env_cfg, mode, 12)
    off, r_off = _rollout_with_order(task, n, env_cfg, "off", 12)
    assert r_on == r_off and r_on > 0
    names = ("obs", "rew", "reset", "root state", "dof state", "progress")
    for k, (a, b) in enumerate(zip(on, off)):
        for name, x, y in zip(names, a, b):
            assert torch.equal(x, y), f"{task} {env_cfg} step {k}: {name} differ with the work order on"


@pytest.mark.parametrize("task,n", [("Ant", 65536), ("MAAnt", 16384)])
def test_sorted_headline_equals_unordered(task, n):
    """The headline configuration runs sorted by default (Ant from 32,768 envs) on the compact 12-wave
    kernel: 8 fused steps at 65,536 envs sorted every launch and unordered give the same obs, rew, reset, root and DOF
    state bit for bit (the sort changes only which envs share a wave).  MA-Ant at 16,384 envs x 4 agents: its env
    units ordered whole."""
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    env_cfg = {"episodeLength": 6}
    on, r_on = _rollout_with_order(task, n, env_cfg, "sort", 8)
    off, r_off = _rollout_with_order(task, n, env_cfg, "off", 8)
    assert r_on == r_off and r_on > 0
    names = ("obs", "rew", "reset", "root state", "dof state", "progress")
    for k, (a, b) in enumerate(zip(on, off)):
        for name, x, y in zip(names, a, b):
            assert torch.equal(x, y), f"{task} {n} step {k}: {name} differ sorted vs unordered"


def _work_order(env, cap):
    """(mode, order, cost) of the env's work ordering through mg_work_order (order: the permutation the last launch
    ran in; cost: the row counts that launch wrote, the next sort's keys)"""
    import ctypes as C
    import numpy as np
    from migym import _abi
    order = np.zeros(cap, np.int32)
    cost = np.zeros(cap, np.uint8)
    mode, n = C.c_int32(-1), C.c_int32(-1)
    _abi.check(env._lib.mg_work_order(env.sim, order.ctypes.data, cost.ctypes.data, cap, C.byref(mode), C.byref(n)),
               env._lib)
    return mode.value, order[:n.value].copy(), cost[:n.value].copy()


@pytest.mark.parametrize("task,n,env_cfg,mode", [("Ant", 65536, {}, None),          # the headline size: sorted by default
                                                 ("Humanoid", 32768, {}, None),     # configs[2]: sorted by default
                                                 ("ShadowHand", 16384, {"objectType": "block"}, None),  # sorted too
                                                 ("Ant", 4099, {}, "sort"),         # 17 ragged sort blocks
                                                 ("MAAnt", 8192, {"numAgents": 4}, "sort")])  # env units of 4 agents
def test_sort_order_is_a_descending_permutation(task, n, env_cfg, mode):
    """The sort mode's counting sort (k_ohist / k_oscatter) at the BASELINE sizes: every launch runs
    its env units in a permutation of 0..units-1 (each unit exactly once) sorted by the previous launch's row counts,
    largest first -- checked exactly on the device's own keys (read before the launch) over 6 launches."""
    import numpy as np
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    old = os.environ.get("MIGYM_ORDER")
    if mode:
        os.environ["MIGYM_ORDER"] = mode
    try:
        cfg = configs.task_config(task, n, sim_device=DEV)
        cfg["env"].update(env_cfg)
        env = migym.make(seed=5, task=task, num_envs=n, sim_device=DEV, rl_device=DEV, headless=True,
                         cfg={"task": cfg})
    finally:
        if old is None:
            os.environ.pop("MIGYM_ORDER", None)
        else:
            os.environ["MIGYM_ORDER"] = old
    units = n
    g = torch.Generator(device=DEV).manual_seed(3)
    prev_cost = None
    for k in range(7):
        a = torch.rand((env.num_actors, env.num_actions), device=DEV, generator=g) * 2 - 1
        env.step(a)
        m, order, cost = _work_order(env, units)
        assert m == 2 and order.size == units and cost.size == units, (m, order.size, units)
        if prev_cost is not None:
            assert np.array_equal(np.sort(order), np.arange(units)), f"launch {k}: not a permutation"
            keys = prev_cost[order].astype(np.int32)
            assert np.all(keys[:-1] >= keys[1:]), f"launch {k}: not in descending row-count order"
            assert keys[0] > 0, "no constraint rows at all: the test would check nothing"
        prev_cost = cost
    env.close()


def test_sorted_step_replays_from_a_captured_graph():
    """The default work ordering holds no host-side state between launches (round 6, ADVICE r5: the totals had
    alternated between two buffers by the host's launch parity, so a graph with an odd number of captured steps
    replayed a sort on uncleared totals and could run one env twice): the step kernel that consumes a sort's
    permutation zeroes the sort's totals.  One sorted Ant step captured in a HIP graph (torch.cuda.graph) and replayed
    five times runs a valid permutation every replay, and its results equal, bit for bit, an unordered twin stepped
    eagerly with the same frozen reset counter.  The in-kernel lists mode refuses capture."""
    import numpy as np
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    n = 4099

    def make(mode):
        old = os.environ.get("MIGYM_ORDER")
        os.environ["MIGYM_ORDER"] = mode
        try:
            cfg = configs.task_config("Ant", n, sim_device=DEV)
            cfg["env"]["episodeLength"] = 5
            return migym.make(seed=11, task="Ant", num_envs=n, sim_device=DEV, rl_device=DEV, headless=True,
                              cfg={"task": cfg})
        finally:
            if old is None:
                os.environ.pop("MIGYM_ORDER", None)
            else:
                os.environ["MIGYM_ORDER"] = old

    env, twin = make("sort"), make("off")
    g = torch.Generator(device=DEV).manual_seed(4)
    a = torch.rand((n, env.num_actions), device=DEV, generator=g) * 2 - 1
    for _ in range(2):   # eager: the second launch is the first sorted one
        env.step(a)
        twin.step(a)
    frozen = env.control_steps
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(device=DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            env.step(a)   # captured, not run
    torch.cuda.current_stream(DEV).wait_stream(side)
    torch.cuda.synchronize()
    for k in range(5):
        graph.replay()
        torch.cuda.synchronize()
        twin.control_steps = frozen   # the graph's frozen reset counter
        twin.step(a)
        torch.cuda.synchronize()
        m, order, _ = _work_order(env, n)
        assert m == 2 and np.array_equal(np.sort(order), np.arange(n)), f"replay {k}: not a permutation"
        for name, x, y in (("obs", env.obs_buf, twin.obs_buf), ("rew", env.rew_buf, twin.rew_buf),
                           ("reset", env.reset_buf, twin.reset_buf), ("root", env.root_states, twin.root_states),
                           ("dof", env.dof_state, twin.dof_state)):
            assert torch.equal(x, y), f"replay {k}: {name} differs from the eager unordered twin"
    lists = make("lists")
    lists.step(a)
    lists.step(a)
    torch.cuda.synchronize()
    graph2 = torch.cuda.CUDAGraph()
    err = None
    try:
        with torch.cuda.stream(side):
            with torch.cuda.graph(graph2, stream=side):
                lists.step(a)
    except Exception as e:   # the refusal (possibly chained behind the graph's own end-of-capture error)
        err = e
    chain, e = "", err
    while e is not None:
        chain += str(e) + " | "
        e = e.__context__
    assert "cannot be captured" in chain, chain
    torch.cuda.synchronize()
    for e in (env, twin, lists):
        e.close()
