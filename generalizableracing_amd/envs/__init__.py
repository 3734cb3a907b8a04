from .racing_cfg import QuadcopterRacingCTBREnvCfg, RacingEnvCfg, training_stage  # noqa: F401


def __getattr__(name):  # lazy: importing the env needs torch + libgr.so
    if name in ("RacingEnv", "RslRlVecEnvWrapper"):
        from . import racing_env

        return getattr(racing_env, name)
    raise AttributeError(name)
