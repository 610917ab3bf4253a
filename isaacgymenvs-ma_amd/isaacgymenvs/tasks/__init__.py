from migym.tasks import isaacgym_task_map, Ant, Humanoid, Cartpole  # noqa: F401
