"""Task configuration defaults and the hydra-free resolver.

The reference composes ``cfg/config.yaml`` + ``cfg/task/<Task>.yaml`` with
hydra/OmegaConf and four custom resolvers (isaacgymenvs/__init__.py:8-11,
35-38).  Neither hydra nor omegaconf is available here, so the values the hot
path reads are restated as plain dicts (same keys, so ``cfg['env'][...]``
overrides written for the reference work unchanged) and interpolations are
resolved eagerly by :func:`task_config`.

Sources of the values: cfg/config.yaml:18-32 (devices, physx threads,
solver), cfg/task/Ant.yaml, Humanoid.yaml, Cartpole.yaml, ShadowHand.yaml.
"""
from __future__ import annotations

import copy
import math

ROOT_DEFAULTS = {
    "physics_engine": "physx",
    "pipeline": "gpu",
    "sim_device": "cuda:0",
    "rl_device": "cuda:0",
    "graphics_device_id": 0,
    "num_threads": 4,
    "solver_type": 1,       # reference default TGS; this build implements PGS
    "num_subscenes": 4,
    "seed": 42,
}

_PHYSX_COMMON = {
    "num_threads": 4, "solver_type": 1, "use_gpu": True, "num_position_iterations": 4,
    "num_velocity_iterations": 0, "contact_offset": 0.02, "rest_offset": 0.0,
    "bounce_threshold_velocity": 0.2, "max_depenetration_velocity": 10.0,
    "default_buffer_size_multiplier": 5.0, "max_gpu_contact_pairs": 8 * 1024 * 1024,
    "num_subscenes": 4, "contact_collection": 0,
}


def _sim(dt=0.0166, **physx):
    p = dict(_PHYSX_COMMON)
    p.update(physx)
    return {"dt": dt, "substeps": 2, "up_axis": "z", "use_gpu_pipeline": True,
            "gravity": [0.0, 0.0, -9.81], "physx": p}


_LOCO_PLANE = {"staticFriction": 1.0, "dynamicFriction": 1.0, "restitution": 0.0}


# task.randomization_params of the task YAMLs (cfg/task/Ant.yaml:63-101, Humanoid.yaml:63-129,
# ShadowHand.yaml:64-169); applied when task.randomize is True (migym/dr.py)
_DR_ANT = {'frequency': 600,
 'observations': {'range': [0, 0.002], 'operation': 'additive', 'distribution': 'gaussian'},
 'actions': {'range': [0.0, 0.02], 'operation': 'additive', 'distribution': 'gaussian'},
 'actor_params': {'ant': {'color': True,
                          'rigid_body_properties': {'mass': {'range': [0.5, 1.5],
                                                             'operation': 'scaling',
                                                             'distribution': 'uniform',
                                                             'setup_only': True}},
                          'dof_properties': {'damping': {'range': [0.5, 1.5],
                                                         'operation': 'scaling',
                                                         'distribution': 'uniform'},
                                             'stiffness': {'range': [0.5, 1.5],
                                                           'operation': 'scaling',
                                                           'distribution': 'uniform'},
                                             'lower': {'range': [0, 0.01],
                                                       'operation': 'additive',
                                                       'distribution': 'gaussian'},
                                             'upper': {'range': [0, 0.01],
                                                       'operation': 'additive',
                                                       'distribution': 'gaussian'}}}}}
_DR_HUMANOID = {'frequency': 600,
 'observations': {'range': [0, 0.002], 'operation': 'additive', 'distribution': 'gaussian'},
 'actions': {'range': [0.0, 0.02], 'operation': 'additive', 'distribution': 'gaussian'},
 'sim_params': {'gravity': {'range': [0, 0.4],
                            'operation': 'additive',
                            'distribution': 'gaussian',
                            'schedule': 'linear',
                            'schedule_steps': 3000}},
 'actor_params': {'humanoid': {'color': True,
                               'rigid_body_properties': {'mass': {'range': [0.5, 1.5],
                                                                  'operation': 'scaling',
                                                                  'distribution': 'uniform',
                                                                  'setup_only': True,
                                                                  'schedule': 'linear',
                                                                  'schedule_steps': 3000}},
                               'rigid_shape_properties': {'friction': {'num_buckets': 500,
                                                                       'range': [0.7, 1.3],
                                                                       'operation': 'scaling',
                                                                       'distribution': 'uniform',
                                                                       'schedule': 'linear',
                                                                       'schedule_steps': 3000},
                                                          'restitution': {'range': [0.0, 0.7],
                                                                          'operation': 'scaling',
                                                                          'distribution': 'uniform',
                                                                          'schedule': 'linear',
                                                                          'schedule_steps': 3000}},
                               'dof_properties': {'damping': {'range': [0.5, 1.5],
                                                              'operation': 'scaling',
                                                              'distribution': 'uniform',
                                                              'schedule': 'linear',
                                                              'schedule_steps': 3000},
                                                  'stiffness': {'range': [0.5, 1.5],
                                                                'operation': 'scaling',
                                                                'distribution': 'uniform',
                                                                'schedule': 'linear',
                                                                'schedule_steps': 3000},
                                                  'lower': {'range': [0, 0.01],
                                                            'operation': 'additive',
                                                            'distribution': 'gaussian',
                                                            'schedule': 'linear',
                                                            'schedule_steps': 3000},
                                                  'upper': {'range': [0, 0.01],
                                                            'operation': 'additive',
                                                            'distribution': 'gaussian',
                                                            'schedule': 'linear',
                                                            'schedule_steps': 3000}}}}}
_DR_SHADOWHAND = {'frequency': 720,
 'observations': {'range': [0, 0.002],
                  'range_correlated': [0, 0.001],
                  'operation': 'additive',
                  'distribution': 'gaussian'},
 'actions': {'range': [0.0, 0.05],
             'range_correlated': [0, 0.015],
             'operation': 'additive',
             'distribution': 'gaussian'},
 'sim_params': {'gravity': {'range': [0, 0.4], 'operation': 'additive', 'distribution': 'gaussian'}},
 'actor_params': {'hand': {'color': True,
                           'tendon_properties': {'damping': {'range': [0.3, 3.0],
                                                             'operation': 'scaling',
                                                             'distribution': 'loguniform'},
                                                 'stiffness': {'range': [0.75, 1.5],
                                                               'operation': 'scaling',
                                                               'distribution': 'loguniform'}},
                           'dof_properties': {'damping': {'range': [0.3, 3.0],
                                                          'operation': 'scaling',
                                                          'distribution': 'loguniform'},
                                              'stiffness': {'range': [0.75, 1.5],
                                                            'operation': 'scaling',
                                                            'distribution': 'loguniform'},
                                              'lower': {'range': [0, 0.01],
                                                        'operation': 'additive',
                                                        'distribution': 'gaussian'},
                                              'upper': {'range': [0, 0.01],
                                                        'operation': 'additive',
                                                        'distribution': 'gaussian'}},
                           'rigid_body_properties': {'mass': {'range': [0.5, 1.5],
                                                              'operation': 'scaling',
                                                              'distribution': 'uniform',
                                                              'setup_only': True}},
                           'rigid_shape_properties': {'friction': {'num_buckets': 250,
                                                                   'range': [0.7, 1.3],
                                                                   'operation': 'scaling',
                                                                   'distribution': 'uniform'}}},
                  'object': {'scale': {'range': [0.95, 1.05],
                                       'operation': 'scaling',
                                       'distribution': 'uniform',
                                       'setup_only': True},
                             'rigid_body_properties': {'mass': {'range': [0.5, 1.5],
                                                                'operation': 'scaling',
                                                                'distribution': 'uniform',
                                                                'setup_only': True}},
                             'rigid_shape_properties': {'friction': {'num_buckets': 250,
                                                                     'range': [0.7, 1.3],
                                                                     'operation': 'scaling',
                                                                     'distribution': 'uniform'}}}}}

TASKS = {
    "Ant": {
        "name": "Ant",
        "env": {
            "numEnvs": 4096, "envSpacing": 5, "episodeLength": 1000, "enableDebugVis": False,
            "clipActions": 1.0, "powerScale": 1.0, "controlFrequencyInv": 1,
            "headingWeight": 0.5, "upWeight": 0.1, "actionsCost": 0.005, "energyCost": 0.05,
            "dofVelocityScale": 0.2, "contactForceScale": 0.1, "jointsAtLimitCost": 0.1,
            "deathCost": -2.0, "terminationHeight": 0.31, "plane": dict(_LOCO_PLANE),
            "asset": {"assetFileName": "mjcf/nv_ant.xml"}, "enableCameraSensors": False,
        },
        "sim": _sim(),
        "task": {"randomize": False, "randomization_params": _DR_ANT},
    },
    "Humanoid": {
        "name": "Humanoid",
        "env": {
            "numEnvs": 4096, "envSpacing": 5, "episodeLength": 1000, "enableDebugVis": False,
            "clipActions": 1.0, "powerScale": 1.0, "headingWeight": 0.5, "upWeight": 0.1,
            "actionsCost": 0.01, "energyCost": 0.05, "dofVelocityScale": 0.1, "angularVelocityScale": 0.25,
            "contactForceScale": 0.01, "jointsAtLimitCost": 0.25, "deathCost": -1.0,
            "terminationHeight": 0.8, "asset": {"assetFileName": "mjcf/nv_humanoid.xml"},
            "plane": dict(_LOCO_PLANE), "enableCameraSensors": False,
        },
        "sim": _sim(),
        "task": {"randomize": False, "randomization_params": _DR_HUMANOID},
    },
    "Cartpole": {
        "name": "Cartpole",
        "env": {
            "numEnvs": 512, "envSpacing": 4.0, "resetDist": 3.0, "maxEffort": 400.0,
            "clipObservations": 5.0, "clipActions": 1.0,
            "asset": {"assetRoot": "../../assets", "assetFileName": "urdf/cartpole.urdf"},
            "enableCameraSensors": False,
        },
        "sim": _sim(rest_offset=0.001, max_depenetration_velocity=100.0, default_buffer_size_multiplier=2.0,
                    max_gpu_contact_pairs=1024 * 1024),
        "task": {"randomize": False},
    },
}

TASKS["ShadowHand"] = {
    "name": "ShadowHand",
    "env": {
        "numEnvs": 16384, "envSpacing": 0.75, "episodeLength": 600, "enableDebugVis": False, "aggregateMode": 1,
        "clipObservations": 5.0, "clipActions": 1.0, "stiffnessScale": 1.0, "forceLimitScale": 1.0,
        "useRelativeControl": False, "dofSpeedScale": 20.0, "actionsMovingAverage": 1.0,
        "controlFrequencyInv": 1, "startPositionNoise": 0.01, "startRotationNoise": 0.0,
        "resetPositionNoise": 0.01, "resetRotationNoise": 0.0, "resetDofPosRandomInterval": 0.2,
        "resetDofVelRandomInterval": 0.0, "forceScale": 0.0, "forceProbRange": [0.001, 0.1],
        "forceDecay": 0.99, "forceDecayInterval": 0.08, "distRewardScale": -10.0, "rotRewardScale": 1.0,
        "rotEps": 0.1, "actionPenaltyScale": -0.0002, "reachGoalBonus": 250, "fallDistance": 0.24,
        "fallPenalty": 0.0, "objectType": "block", "observationType": "full_state",
        "asymmetric_observations": False, "successTolerance": 0.1, "printNumSuccesses": False,
        "maxConsecutiveSuccesses": 0,
        "asset": {"assetFileName": "mjcf/open_ai_assets/hand/shadow_hand.xml",
                  "assetFileNameBlock": "urdf/objects/cube_multicolor.urdf",
                  "assetFileNameEgg": "mjcf/open_ai_assets/hand/egg.xml",
                  "assetFileNamePen": "mjcf/open_ai_assets/hand/pen.xml"},
        "enableCameraSensors": False,
    },
    "sim": _sim(dt=0.01667, num_position_iterations=8, contact_offset=0.002, rest_offset=0.0,
                bounce_threshold_velocity=0.2, max_depenetration_velocity=1000.0),
    "task": {"randomize": False, "randomization_params": _DR_SHADOWHAND},
}

# Multi-agent Ant (build-defined, SURVEY.md §8(a) row A-MA): A ant actors per env.
TASKS["MAAnt"] = copy.deepcopy(TASKS["Ant"])
TASKS["MAAnt"]["name"] = "MAAnt"
TASKS["MAAnt"]["env"].update({"numAgents": 4, "agentSpacing": 2.0})


def resolve_default(default, arg):
    """``${resolve_default:d,x}`` (isaacgymenvs/__init__.py:11)."""
    return default if arg in ("", None) else arg


def task_config(task: str, num_envs=None, sim_device="cuda:0", pipeline="gpu", overrides=None) -> dict:
    """cfg.task as a plain dict with interpolations resolved (``omegaconf_to_dict``)."""
    if task not in TASKS:
        raise ValueError(f"unknown task {task!r}; available: {sorted(TASKS)}")
    cfg = copy.deepcopy(TASKS[task])
    cfg["physics_engine"] = ROOT_DEFAULTS["physics_engine"]
    cfg["env"]["numEnvs"] = resolve_default(cfg["env"]["numEnvs"], num_envs)
    cfg["sim"]["use_gpu_pipeline"] = pipeline.lower() == "gpu"                   # ${eq:${...pipeline},"gpu"}
    cfg["sim"]["physx"]["use_gpu"] = "cuda" in sim_device.lower()                 # ${contains:"cuda",...}
    for k, v in (overrides or {}).items():
        node = cfg
        parts = k.split(".")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = v
    return cfg


def clip_value(cfg_env, key):
    v = cfg_env.get(key, math.inf)
    return float(v)
