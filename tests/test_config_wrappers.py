"""CPU tests of the hydra-free YAML composition (isaacgymenvs/__init__.py:8-11 resolvers, cfg/config.yaml +
cfg/task/<Task>.yaml) and of the rl_games wrappers (rlgames_utils.py:242-424) on a stand-in env.

The synthetic YAMLs below are written by the tests; where the reference's own ``cfg/`` tree is present
(the build container), its four task YAMLs composed by the loader must equal migym.configs' restated
defaults exactly.
"""
import os

import numpy as np
import pytest
import torch

from migym import configs, yaml_config as Y
from migym.spaces import Box
from migym.utils.rlgames_utils import ComplexObsRLGPUEnv, RLGPUEnv, register_env_creator

REF_CFG = "/root/reference/isaacgymenvs/cfg"

ROOT_YAML = """
task_name: ${task.name}
num_envs: ''
seed: 42
pipeline: 'gpu'
sim_device: 'cuda:0'
physics_engine: 'physx'
num_threads: 4
solver_type: 1
label: run-${task.name}-${seed}
wandb_name: ${train.params.config.name}
defaults:
  - task: Toy
  - _self_
"""

TASK_YAML = """
name: Toy
physics_engine: ${..physics_engine}
env:
  numEnvs: ${resolve_default:4096,${...num_envs}}
  episodeLength: 1000
  useGpu: ${contains:"cuda",${...sim_device}}
  mode: ${if:${eq:${...pipeline},"GPU"},fast,slow}
  spacing: ${.episodeLength}
sim:
  use_gpu_pipeline: ${eq:${...pipeline},"gpu"}
  physx:
    num_threads: ${....num_threads}
    solver_type: ${....solver_type}
    use_gpu: ${contains:"cuda",${....sim_device}}
"""


@pytest.fixture()
def cfg_dir(tmp_path):
    (tmp_path / "task").mkdir()
    (tmp_path / "config.yaml").write_text(ROOT_YAML)
    (tmp_path / "task" / "Toy.yaml").write_text(TASK_YAML)
    (tmp_path / "task" / "Cyc.yaml").write_text("name: Cyc\na: ${.b}\nb: ${.a}\n")
    (tmp_path / "task" / "Bad.yaml").write_text("name: Bad\na: ${nope.x}\n")
    return str(tmp_path)


def test_resolvers_and_relative_interpolation(cfg_dir):
    c = Y.compose(cfg_dir)
    t = c["task"]
    assert c["task_name"] == "Toy"
    assert c["label"] == "run-Toy-42"                     # string interpolation keeps the text around it
    assert c["wandb_name"] == "${train.params.config.name}"  # unresolvable outside the task group: kept (lazy)
    assert t["physics_engine"] == "physx"
    assert t["env"]["numEnvs"] == 4096                    # resolve_default: '' -> the default
    assert t["env"]["useGpu"] is True                     # contains
    assert t["env"]["mode"] == "fast"                     # if(eq) with case-insensitive eq
    assert t["env"]["spacing"] == 1000                    # one dot: a sibling, typed
    assert t["sim"]["use_gpu_pipeline"] is True
    assert t["sim"]["physx"]["num_threads"] == 4 and t["sim"]["physx"]["solver_type"] == 1


def test_overrides(cfg_dir):
    c = Y.compose(cfg_dir, overrides=["num_envs=64", "sim_device=cpu", "pipeline=cpu", "task.env.episodeLength=7",
                                      "seed=3"])
    t = c["task"]
    assert t["env"]["numEnvs"] == 64
    assert t["env"]["useGpu"] is False and t["sim"]["physx"]["use_gpu"] is False
    assert t["sim"]["use_gpu_pipeline"] is False and t["env"]["mode"] == "slow"
    assert t["env"]["spacing"] == 7
    assert c["label"] == "run-Toy-3"
    tc = Y.task_config_from_yaml("Toy", cfg_dir, num_envs=12, sim_device="cuda:1")
    assert tc["env"]["numEnvs"] == 12 and tc["env"]["useGpu"] is True


def test_errors(cfg_dir):
    with pytest.raises(Y.ConfigError, match="cycle"):
        Y.compose(cfg_dir, task="Cyc")
    with pytest.raises(Y.ConfigError, match="not found"):
        Y.compose(cfg_dir, task="Bad")
    with pytest.raises(Y.ConfigError, match="no task config"):
        Y.compose(cfg_dir, task="Missing")


def test_single_task_file(tmp_path):
    p = tmp_path / "Toy.yaml"
    p.write_text(TASK_YAML)
    t = Y.task_config_from_file(str(p), num_envs=32)
    assert t["env"]["numEnvs"] == 32 and t["sim"]["physx"]["use_gpu"] is True


@pytest.mark.skipif(not os.path.isdir(REF_CFG), reason="the reference's cfg/ tree is only in the build container")
@pytest.mark.parametrize("task", ["Ant", "Humanoid", "Cartpole", "ShadowHand"])
@pytest.mark.parametrize("dev,pipe", [("cuda:0", "gpu"), ("cpu", "cpu")])
def test_reference_yamls_equal_builtin_defaults(task, dev, pipe):
    a = Y.task_config_from_yaml(task, REF_CFG, num_envs=128, sim_device=dev, pipeline=pipe)
    b = configs.task_config(task, 128, sim_device=dev, pipeline=pipe)
    assert a == b


class FakeEnv:
    """obs_dict {'obs', 'states'} like the tasks' step / reset (no GPU needed)."""

    num_states = 5
    num_agents = 1

    def __init__(self, n=4):
        self.n = n
        self.observation_space = Box(np.full(7, -np.inf), np.full(7, np.inf))
        self.state_space = Box(np.full(5, -np.inf), np.full(5, np.inf))
        self.action_space = Box(np.full(2, -1.0), np.full(2, 1.0))
        self.frames = None
        self.state = None

    def _obs(self):
        return {"obs": torch.arange(self.n * 7, dtype=torch.float32).view(self.n, 7),
                "states": -torch.arange(self.n * 5, dtype=torch.float32).view(self.n, 5)}

    def step(self, a):
        return self._obs(), torch.zeros(self.n), torch.zeros(self.n, dtype=torch.long), {}

    def reset(self):
        return self._obs()

    def set_train_info(self, f):
        self.frames = f

    def get_env_state(self):
        return {"x": 1}

    def set_env_state(self, s):
        self.state = s


def test_complex_obs_wrapper_concat_and_dict():
    register_env_creator("fake", lambda **kw: FakeEnv(**kw))
    spec = {"obs": {"names": ["obs", "states"], "concat": True, "space_name": "observation_space"},
            "states": {"names": ["states"], "concat": False, "space_name": "state_space"}}
    w = ComplexObsRLGPUEnv("fake", 1, spec, n=3)
    o = w.reset()
    assert o["obs"].shape == (3, 12)
    assert torch.equal(o["obs"][:, 7:], w.env._obs()["states"])
    assert set(o["states"].keys()) == {"states"}
    o2, r, d, info = w.step(torch.zeros(3, 2))
    assert torch.equal(o2["obs"], o["obs"])
    info = w.get_env_info()
    assert info["observation_space"].shape == (12,)
    assert info["state_space"]["states"].shape == (5,)
    assert w.get_number_of_agents() == 1
    w.set_train_info(10)
    assert w.env.frames == 10
    assert w.get_env_state() == {"x": 1}
    w.set_env_state({"y": 2})
    assert w.env.state == {"y": 2}
    with pytest.raises(ValueError):
        ComplexObsRLGPUEnv("fake", 1, {}, n=3)


def test_rlgpu_env_registry_and_positional_env():
    register_env_creator("fake2", lambda **kw: FakeEnv(**kw))
    w = RLGPUEnv("fake2", 1, n=2)
    assert w.get_env_info()["state_space"].shape == (5,)
    e = FakeEnv()
    assert RLGPUEnv(e).env is e
    with pytest.raises(KeyError):
        RLGPUEnv("nope", 1)
