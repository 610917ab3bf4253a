from migym.utils.rlgames_utils import (ComplexObsRLGPUEnv, RLGPUEnv, env_configurations,  # noqa: F401
                                     get_rlgames_env_creator, register_env_creator)
