"""Drop-in env package: `from envs.vss import VSS`, `from envs.wrappers import make_env`."""
