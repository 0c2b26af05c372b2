"""Experiment configuration resolution (reference: ``src/orion/core/io/resolve_config.py:61-288``).

Precedence, lowest to highest: **defaults < env vars < database < ``--config`` file < cmdargs <
metadata**.  Defaults: ``max_trials=inf``, ``worker_trials=inf``, ``pool_size=1``,
``algorithms='random'``, database options from the global configuration.

``fetch_metadata`` records ``user``, ``orion_version``, ``user_script`` (absolute when executable),
``user_args`` and, when the script lives in a git repository, ``VCS`` = ``{type, is_dirty,
HEAD_sha, active_branch, diff_sha}`` -- computed with the ``git`` CLI (the reference needs
gitpython).
"""
from __future__ import annotations

import errno
import getpass
import hashlib
import logging
import os
import subprocess

import yaml

from .. import __version__
from ..core.config import config as global_config

log = logging.getLogger(__name__)

INF = float("inf")
DEF_CMD_MAX_TRIALS = (INF, "inf/until preempted")
DEF_CMD_WORKER_TRIALS = (INF, "inf/until preempted")
DEF_CMD_POOL_SIZE = (1, "1")

ENV_VARS_DB = [("MOPT_DB_NAME", "name"), ("MOPT_DB_TYPE", "type"), ("MOPT_DB_ADDRESS", "host"),
               ("MOPT_DB_PORT", "port"), ("ORION_DB_NAME", "name"), ("ORION_DB_TYPE", "type"),
               ("ORION_DB_ADDRESS", "host"), ("ORION_DB_PORT", "port")]
ENV_VARS = dict(database=ENV_VARS_DB)


def is_exe(path: str) -> bool:
    return os.path.isfile(path) and os.access(path, os.X_OK)


def get_user() -> str:
    try:
        return getpass.getuser()
    except Exception:  # pragma: no cover - no passwd entry
        return os.environ.get("USER", "unknown")


def fetch_config(args: dict) -> dict:
    """The YAML given with ``--config`` (a path or an open file)."""
    cfg_file = args.get("config")
    if not cfg_file:
        return {}
    if hasattr(cfg_file, "read"):
        cfg_file.seek(0)
        data = yaml.safe_load(cfg_file)
    else:
        with open(cfg_file) as f:
            data = yaml.safe_load(f)
    return data or {}


def fetch_default_options() -> dict:
    out = {"name": None, "user": get_user(), "max_trials": DEF_CMD_MAX_TRIALS[0],
           "worker_trials": DEF_CMD_WORKER_TRIALS[0], "pool_size": DEF_CMD_POOL_SIZE[0],
           "algorithms": "random"}
    out["database"] = {k: global_config.database[k] for k in ("name", "type", "host", "port")}
    return out


def fetch_env_vars() -> dict:
    env = {}
    for signif, evars in ENV_VARS.items():
        env[signif] = {}
        for var, key in evars:
            v = os.getenv(var)
            if v is not None and key not in env[signif]:
                env[signif][key] = v
    return env


def _git(repo_dir, *args):
    return subprocess.run(["git", "-C", repo_dir, *args], capture_output=True, text=True,
                          timeout=30)


def infer_versioning_metadata(user_script: str) -> dict:
    """git metadata of the repository holding ``user_script`` ({} outside a repository)."""
    d = os.path.dirname(os.path.abspath(user_script))
    try:
        top = _git(d, "rev-parse", "--show-toplevel")
    except (OSError, subprocess.SubprocessError):
        return {}
    if top.returncode != 0:
        log.warning("Script %s is not in a git repository. Code modification won't be detected.",
                    os.path.abspath(user_script))
        return {}
    head = _git(d, "rev-parse", "HEAD")
    if head.returncode != 0:  # repository without commits
        return {}
    status = _git(d, "status", "--porcelain", "--untracked-files=no")
    branch = _git(d, "symbolic-ref", "--short", "-q", "HEAD")
    diff = _git(d, "diff", "HEAD")
    return {"type": "git", "is_dirty": bool(status.stdout.strip()), "HEAD_sha": head.stdout.strip(),
            "active_branch": branch.stdout.strip() or None,
            "diff_sha": hashlib.sha256(diff.stdout.encode("utf-8")).hexdigest()}


def fetch_metadata(cmdargs: dict) -> dict:
    md = {"orion_version": __version__}
    user_args = list(cmdargs.get("user_args") or [])
    if len(user_args) == 1 and user_args[0] == "":
        user_args = []
    user_script = user_args[0] if user_args else None
    if user_script:
        abs_script = os.path.abspath(user_script)
        if is_exe(abs_script):
            user_script = abs_script
    if user_script and not os.path.exists(user_script):
        raise OSError(errno.ENOENT, "The path specified for the script does not exist", user_script)
    if user_script:
        md["user_script"] = user_script
        md["VCS"] = infer_versioning_metadata(user_script)
    if user_args:
        md["user_args"] = user_args[1:]
    md["user"] = get_user()
    return md


def merge_configs(*configs) -> dict:
    """Right-most wins; dicts merge recursively; ``None`` never overwrites."""
    merged = configs[0]
    for cfg in configs[1:]:
        for key, value in cfg.items():
            if isinstance(value, dict) and isinstance(merged.get(key), dict):
                merged[key] = merge_configs(merged[key], value)
            elif value is not None:
                merged[key] = value
    return merged
