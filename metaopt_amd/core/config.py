"""Typed, layered configuration (reference: ``src/orion/core/io/config.py:32-268`` and the global
schema of ``src/orion/core/__init__.py:44-111``).

Precedence for every option: **explicit value > environment variable > YAML file > default**.
Options are declared with :meth:`Configuration.add_option`; sub-configurations nest
(``config.database.host``) and dotted item access works (``config['database.host']``).

Global schema (``config``):
  * ``database.{name,type,host,port}`` -- env ``MOPT_DB_NAME/TYPE/ADDRESS/PORT`` (the reference's
    ``ORION_DB_*`` names are honoured too);
  * ``worker.{heartbeat=120, max_broken=3, max_idle_time=60, pacemaker_interval=60}``;
  * ``device.{gpus, population_per_gpu, dtype}`` -- the device data plane;
  * ``user_script_config='config'`` -- the user-script argument that names its config file.
Global YAML files: ``/etc/xdg/mopt/mopt_config.yaml`` and ``~/.config/mopt/mopt_config.yaml``.
"""
from __future__ import annotations

import logging
import os
from typing import Any, Callable, Optional

import yaml

from ..utils.flatten import flatten

log = logging.getLogger(__name__)

NOT_SET = object()


class ConfigurationError(Exception):
    pass


def _bool(v):
    if isinstance(v, str):
        return v.strip().lower() in ("1", "true", "yes", "on")
    return bool(v)


class Configuration:
    """Options with precedence value > env var > yaml > default."""

    SPECIAL_KEYS = ["_config", "_yaml", "_default", "_env_var", "_value"]

    def __init__(self):
        object.__setattr__(self, "_config", {})
        object.__setattr__(self, "_subconfigs", {})

    # -- definition ---------------------------------------------------------------------------
    def add_option(self, key: str, option_type: Callable, default: Any = NOT_SET,
                   env_var=None):
        if key in self._config or key in self._subconfigs:
            raise ValueError(f"Configuration already has {key}")
        if option_type is bool:
            option_type = _bool
        setting = {"type": option_type}
        if default is not NOT_SET:
            setting["default"] = default
        if env_var:
            setting["env_var"] = [env_var] if isinstance(env_var, str) else list(env_var)
        self._config[key] = setting

    # -- lookup -------------------------------------------------------------------------------
    def __getattr__(self, key):
        if key.startswith("__"):
            raise AttributeError(key)
        subs = object.__getattribute__(self, "_subconfigs")
        if key in subs:
            return subs[key]
        cfg = object.__getattribute__(self, "_config")
        if key not in cfg:
            raise ConfigurationError(f"Configuration does not have an attribute '{key}'.")
        s = cfg[key]
        if "value" in s:
            value = s["value"]
        elif any(e in os.environ for e in s.get("env_var", [])):
            value = next(os.environ[e] for e in s["env_var"] if e in os.environ)
        elif "yaml" in s:
            value = s["yaml"]
        elif "default" in s:
            value = s["default"]
        else:
            raise ConfigurationError(f"Configuration not set and no default provided: {key}.")
        return s["type"](value) if value is not None else None

    def __setattr__(self, key, value):
        if key in self._config:
            self._validate(key, value)
            self._config[key]["value"] = value
        elif isinstance(value, Configuration):
            self._subconfigs[key] = value
        else:
            raise TypeError(f"Can only set {key} as a Configuration, not {type(value)}. Use "
                            "add_option to set a new option.")

    def _validate(self, key, value):
        if isinstance(value, Configuration):
            raise TypeError(f"Cannot overwrite option {key} with a configuration")
        try:
            if value is not None:
                self._config[key]["type"](value)
        except (ValueError, TypeError) as exc:
            raise TypeError(f"Option {key} of type {self._config[key]['type']} cannot be set to "
                            f"{value} with type {type(value)}") from exc

    def __setitem__(self, key, value):
        keys = key.split(".")
        if len(keys) == 2 and ("_" + keys[1].lstrip("_")) in self.SPECIAL_KEYS and \
                keys[0] in self._config:
            self._validate(keys[0], value)
            self._config[keys[0]][keys[1].lstrip("_")] = value
        elif len(keys) == 1:
            setattr(self, keys[0], value)
        else:
            sub = getattr(self, keys[0])
            sub[".".join(keys[1:])] = value

    def __getitem__(self, key):
        keys = key.split(".")
        if len(keys) > 1:
            return getattr(self, keys[0])[".".join(keys[1:])]
        return getattr(self, keys[0])

    def __contains__(self, key):
        keys = key.split(".")
        if len(keys) > 1:
            return keys[0] in self._subconfigs and ".".join(keys[1:]) in self._subconfigs[keys[0]]
        return key in self._config or key in self._subconfigs

    def unset(self, key):
        """Drop an explicitly set value (fall back to env/yaml/default)."""
        keys = key.split(".")
        if len(keys) > 1:
            return getattr(self, keys[0]).unset(".".join(keys[1:]))
        self._config[key].pop("value", None)

    # -- files --------------------------------------------------------------------------------
    def load_yaml(self, path: str) -> None:
        with open(path) as f:
            cfg = yaml.safe_load(f)
        if cfg is None:
            return
        for key, value in flatten(cfg).items():
            self[key]  # raises for unknown options
            self[key + "._yaml"] = value

    def to_dict(self) -> dict:
        out = {}
        for k in self._config:
            try:
                out[k] = getattr(self, k)
            except ConfigurationError:
                pass
        for k, sub in self._subconfigs.items():
            out[k] = sub.to_dict()
        return out

    def defaults(self) -> dict:
        out = {k: s.get("default") for k, s in self._config.items()}
        for k, sub in self._subconfigs.items():
            out[k] = sub.defaults()
        return out

    def env_vars(self) -> dict:
        """{option: value} for options currently overridden by environment variables."""
        out = {}
        for k, s in self._config.items():
            for e in s.get("env_var", []):
                if e in os.environ:
                    out[k] = s["type"](os.environ[e])
                    break
        for k, sub in self._subconfigs.items():
            d = sub.env_vars()
            if d:
                out[k] = d
        return out


def user_config_dir() -> str:
    base = os.environ.get("XDG_CONFIG_HOME") or os.path.join(os.path.expanduser("~"), ".config")
    return os.path.join(base, "mopt")


DEF_CONFIG_FILES_PATHS = [
    os.path.join("/etc", "xdg", "mopt", "mopt_config.yaml"),
    os.path.join(user_config_dir(), "mopt_config.yaml"),
]


def define_config() -> Configuration:
    config = Configuration()

    db = Configuration()
    db.add_option("name", str, "mopt", env_var=["MOPT_DB_NAME", "ORION_DB_NAME"])
    db.add_option("type", str, "PickledDB", env_var=["MOPT_DB_TYPE", "ORION_DB_TYPE"])
    db.add_option("host", str, "", env_var=["MOPT_DB_ADDRESS", "ORION_DB_ADDRESS"])
    db.add_option("port", int, 27017, env_var=["MOPT_DB_PORT", "ORION_DB_PORT"])
    config.database = db

    worker = Configuration()
    worker.add_option("heartbeat", int, 120, env_var="MOPT_HEARTBEAT")
    worker.add_option("max_broken", int, 3, env_var="MOPT_MAX_BROKEN")
    worker.add_option("max_idle_time", int, 60, env_var="MOPT_MAX_IDLE_TIME")
    worker.add_option("pacemaker_interval", int, 60, env_var="MOPT_PACEMAKER_INTERVAL")
    config.worker = worker

    device = Configuration()
    device.add_option("gpus", int, 1, env_var="MOPT_GPUS")
    device.add_option("population_per_gpu", int, 256, env_var="MOPT_POPULATION_PER_GPU")
    device.add_option("dtype", str, "bf16", env_var="MOPT_DTYPE")
    config.device = device

    config.add_option("user_script_config", str, "config")
    return config


def build_config(paths=None) -> Configuration:
    cfg = define_config()
    for path in (DEF_CONFIG_FILES_PATHS if paths is None else paths):
        if os.path.exists(path):
            try:
                cfg.load_yaml(path)
            except Exception as exc:  # pragma: no cover - bad user file
                log.warning("ignoring global config %s: %s", path, exc)
    return cfg


config = build_config()
