from migym.utils.rlgames_utils import RLGPUEnv, get_rlgames_env_creator  # noqa: F401
