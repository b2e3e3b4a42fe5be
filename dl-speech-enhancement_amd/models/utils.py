"""models/utils.py (reference :13-15)."""


def check_mode(mode, method):
    if mode not in ("causal",):
        raise AssertionError(f"Mode {mode} does not support {method}!")
