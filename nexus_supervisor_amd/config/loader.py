"""Layered configuration loader (replaces nexus-core ``configurations.LoadConfig[T]``,
called at ``/root/reference/main.go:14``).

Precedence (lowest → highest):

1. schema defaults (= Helm defaults, ``/root/reference/.helm/values.yaml``)
2. ``appconfig.yaml`` (cwd, or ``$NEXUS_CONFIG_DIR`` / explicit ``path``)
3. ``appconfig.<APPLICATION_ENVIRONMENT>.yaml`` overlay (``appconfig.local.yaml``
   exists in the reference; ``APPLICATION_ENVIRONMENT=units`` in its CI,
   ``/root/reference/.github/workflows/build.yaml:54``)
4. ``NEXUS__`` environment: kebab keys → UPPER_SNAKE, nesting with ``__``
   (``NEXUS__RATE_LIMIT_ELEMENTS_PER_SECOND``,
   ``NEXUS__SCYLLA_CQL_STORE__HOSTS`` — ``/root/reference/.helm/templates/deployment.yaml:49-66``).

Empty strings in YAML (the reference ships every key as ``""``) mean "unset" and
keep the default rather than decoding to zero.
"""
from __future__ import annotations

import dataclasses
import logging
import os
from typing import Any, Dict, Mapping, Optional, get_type_hints

import yaml

from ..utils.durations import parse_duration
from .schema import ConfigError, SupervisorConfig, validate

ENV_PREFIX = "NEXUS__"
_TRUE = {"1", "true", "yes", "on", "y", "t"}
_FALSE = {"0", "false", "no", "off", "n", "f"}


def env_name(path) -> str:
    """``("scylla-cql-store", "hosts")`` → ``NEXUS__SCYLLA_CQL_STORE__HOSTS``."""
    return ENV_PREFIX + "__".join(p.replace("-", "_").upper() for p in path)


def _coerce(value: Any, ftype, kind: Optional[str], key: str):
    try:
        if kind == "duration":
            return parse_duration(value)
        if kind == "list":
            if isinstance(value, str):
                return [v.strip() for v in value.split(",") if v.strip()]
            if value is None:
                return []
            return [str(v) for v in value]
        if kind == "number":
            return float(value)
        if ftype is bool:
            if isinstance(value, bool):
                return value
            s = str(value).strip().lower()
            if s in _TRUE:
                return True
            if s in _FALSE:
                return False
            raise ValueError(value)
        if ftype is int:
            if isinstance(value, bool):
                raise ValueError(value)
            if isinstance(value, float) and not value.is_integer():
                raise ValueError(value)
            return int(str(value).strip()) if isinstance(value, str) else int(value)
        if ftype is float:
            return float(value)
        if ftype is str:
            return "" if value is None else str(value)
    except (TypeError, ValueError) as e:
        raise ConfigError(f"invalid value for {key!r}: {value!r}") from e
    return value


def _is_unset(value) -> bool:
    return value is None or (isinstance(value, str) and value.strip() == "")


def _apply(obj, data: Mapping[str, Any], env: Mapping[str, str], path=(), unknown: Optional[list] = None):
    """Fill ``obj`` from ``data`` + env.  Unknown keys raise, or are collected into
    ``unknown`` (dotted paths) when a list is given."""
    hints = get_type_hints(type(obj))
    known = set()
    for f in dataclasses.fields(obj):
        key = f.metadata["key"]
        known.add(key)
        fpath = path + (key,)
        ftype = hints[f.name]
        sub = getattr(obj, f.name)
        if dataclasses.is_dataclass(sub):
            sub_data = data.get(key) if isinstance(data, Mapping) else None
            _apply(sub, sub_data if isinstance(sub_data, Mapping) else {}, env, fpath, unknown)
            continue
        kind = f.metadata.get("kind")
        if isinstance(data, Mapping) and key in data and not (_is_unset(data[key]) and kind != "list"):
            val = data[key]
            if not (kind == "list" and val in ("", None)):
                setattr(obj, f.name, _coerce(val, ftype, kind, ".".join(fpath)))
        ev = env.get(env_name(fpath))
        if ev is not None and ev.strip() != "":
            setattr(obj, f.name, _coerce(ev, ftype, kind, env_name(fpath)))
    if isinstance(data, Mapping):
        extra = set(data) - known
        if extra and unknown is None:
            raise ConfigError(f"unknown config keys at {'.'.join(path) or '<root>'}: {sorted(extra)}")
        if extra:
            unknown.extend(".".join(path + (k,)) for k in sorted(extra))


def _read_yaml(path: str) -> Dict[str, Any]:
    with open(path, "r", encoding="utf-8") as fh:
        data = yaml.safe_load(fh) or {}
    if not isinstance(data, dict):
        raise ConfigError(f"{path}: top-level YAML must be a mapping")
    return data


def _deep_merge(base: Dict[str, Any], over: Mapping[str, Any]) -> Dict[str, Any]:
    out = dict(base)
    for k, v in over.items():
        if isinstance(v, Mapping) and isinstance(out.get(k), Mapping):
            out[k] = _deep_merge(out[k], v)
        elif _is_unset(v) and k in out:
            continue
        else:
            out[k] = v
    return out


def load_config(
    path: Optional[str] = None,
    env: Optional[Mapping[str, str]] = None,
    overrides: Optional[Mapping[str, Any]] = None,
    do_validate: bool = True,
) -> SupervisorConfig:
    """Load a :class:`SupervisorConfig` from defaults, YAML files and ``NEXUS__`` env.

    ``overrides`` is a kebab-keyed mapping applied after the files (tests use it).
    Unknown keys are logged and ignored, as viper does for the reference (an appconfig
    with keys of a newer or older release still starts); ``NEXUS_CONFIG_STRICT=1`` makes
    them fatal.
    """
    env = os.environ if env is None else env
    data: Dict[str, Any] = {}
    if path is None:
        cfg_dir = env.get("NEXUS_CONFIG_DIR", os.getcwd())
        candidate = os.path.join(cfg_dir, "appconfig.yaml")
        path = candidate if os.path.exists(candidate) else None
    if path:
        data = _read_yaml(path)
        app_env = env.get("APPLICATION_ENVIRONMENT", "").strip()
        if app_env:
            overlay = os.path.join(os.path.dirname(os.path.abspath(path)), f"appconfig.{app_env}.yaml")
            if os.path.exists(overlay):
                data = _deep_merge(data, _read_yaml(overlay))
    if overrides:
        data = _deep_merge(data, overrides)
    cfg = SupervisorConfig()
    strict = str(env.get("NEXUS_CONFIG_STRICT", "")).strip().lower() in _TRUE
    unknown: list = []
    _apply(cfg, data, env, unknown=None if strict else unknown)
    if unknown:
        logging.getLogger("nexus_supervisor_amd.config").warning(
            "ignoring unknown config keys (set NEXUS_CONFIG_STRICT=1 to refuse them): %s", ", ".join(unknown))
    return validate(cfg) if do_validate else cfg


def iter_keys(cls=SupervisorConfig, path=()):
    """Yield ``(key_path, env_name, default, field)`` for every leaf key (docs + tests)."""
    inst = cls()
    for f in dataclasses.fields(inst):
        fpath = path + (f.metadata["key"],)
        sub = getattr(inst, f.name)
        if dataclasses.is_dataclass(sub):
            yield from iter_keys(type(sub), fpath)
        else:
            yield fpath, env_name(fpath), sub, f


def to_mapping(cfg) -> Dict[str, Any]:
    """Config as a kebab-keyed dict, secrets included (hand-off to worker processes)."""
    out: Dict[str, Any] = {}
    for f in dataclasses.fields(cfg):
        v = getattr(cfg, f.name)
        out[f.metadata["key"]] = to_mapping(v) if dataclasses.is_dataclass(v) else (list(v) if isinstance(v, list) else v)
    return out


def from_mapping(data: Mapping[str, Any], do_validate: bool = True) -> SupervisorConfig:
    """Inverse of :func:`to_mapping` (no files, no environment)."""
    cfg = SupervisorConfig()
    _apply(cfg, data, {})
    return validate(cfg) if do_validate else cfg


def redacted(cfg) -> Dict[str, Any]:
    """Config as a kebab-keyed dict with secrets masked (for the startup log line)."""
    out: Dict[str, Any] = {}
    for f in dataclasses.fields(cfg):
        v = getattr(cfg, f.name)
        if dataclasses.is_dataclass(v):
            out[f.metadata["key"]] = redacted(v)
        elif f.metadata.get("secret") and v:
            out[f.metadata["key"]] = "***"
        else:
            out[f.metadata["key"]] = v
    return out
