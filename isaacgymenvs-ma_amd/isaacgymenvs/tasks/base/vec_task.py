from migym.tasks.base.vec_task import Env, VecTask  # noqa: F401
