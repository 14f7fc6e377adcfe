"""The exporter configuration, as seen from Python: a view of the native options.

Keys, defaults, value coercion, the flag vocabulary, the precedence (defaults < YAML file <
environment < ``--compat`` < flags), the host-name fallback and the CRI socket autodetect are
implemented ONCE, in C++ (csrc/core/options.cpp, the table behind ``bin/gpumon-exporter``). This
module wraps that object so ``gpumon serve`` and the tools read exactly what the DaemonSet's
native entry point reads (two parsers had drifted).

Reference configuration (/root/reference/gpu.py:17-26, gpu_monitor.yaml:29-37):
  * ``NODE_NAME``    — node name tag; the reference's ``"no_name"`` fallback never reached its lines
    (quirk Q1). Here: NODE_NAME, then the host name, then ``"no_name"``.
  * ``INFLUXDB_URL`` — when set, the Influx compat push is enabled (batched, one POST per tick).
  * the 10 s sleep (gpu.py:263) -> ``interval`` (default 1 s); the opt-in docker label
    mlgpu=mlgpu (gpu.py:186-188) -> ``opt_in_label`` (``--compat`` sets it and the 10 s interval).
"""

from __future__ import annotations

import argparse
import json
import logging
import os
from typing import Any, Dict, List, Optional

from ._native import core


class ConfigError(ValueError):
    """A configuration the exporter cannot run with (the CLI exits 2 with the message)."""


class Config:
    """Mutable configuration backed by a native ``Options`` object.

    ``Config(interval=0.1, devices=[0])`` / ``cfg.interval`` / ``cfg.apply_dict({...})`` /
    ``cfg.apply_env(env)`` read and write the native keys; an unknown key raises ValueError, a bad
    value ConfigError. ``finalized()`` resolves what the exporter is started with."""

    __slots__ = ("_o",)

    def __init__(self, _options=None, **kw):
        object.__setattr__(self, "_o", _options if _options is not None else core().Options())
        self.apply_dict(kw)

    # ------------------------------------------------------------------ keys
    def _set(self, key: str, value: Any) -> None:
        try:
            self._o.set(key, value)
        except KeyError:
            raise ValueError(f"unknown config key: {key}") from None
        except ValueError as e:
            raise ConfigError(str(e)) from None

    def to_dict(self, redact: bool = False) -> Dict[str, Any]:
        return json.loads(self._o.to_json(redact))

    def __getattr__(self, name: str) -> Any:
        if name.startswith("__"):
            raise AttributeError(name)
        d = self.to_dict()
        if name in d:
            return d[name]
        raise AttributeError(name)

    def __setattr__(self, name: str, value: Any) -> None:
        self._set(name, value)

    def __repr__(self) -> str:
        return f"Config({self.to_dict(redact=True)})"

    def copy(self) -> "Config":
        return Config(self._o.copy())

    # ------------------------------------------------------------------ sources
    def apply_dict(self, d: Optional[Dict[str, Any]]) -> "Config":
        for k, v in (d or {}).items():
            self._set(k.replace("-", "_"), v)
        return self

    def apply_env(self, env: Optional[Dict[str, str]] = None) -> "Config":
        """NODE_NAME, INFLUXDB_URL / _TOKEN and GPUMON_<KEY>; a GPUMON_ name that is neither a key
        nor an environment-only variable (a typo) is logged and ignored, as the binary does."""
        try:
            unknown = self._o.apply_env(dict(os.environ if env is None else env))
        except ValueError as e:
            raise ConfigError(str(e)) from None
        for k in unknown or []:
            logging.getLogger("gpumon").warning(
                "environment: %s is neither a configuration key nor a GPUMON_ variable (ignored)", k)
        return self

    def apply_file(self, path: str) -> List[str]:
        """A YAML config file (the ConfigMap format); returns the keys it does not know."""
        try:
            return list(self._o.load_file(path))
        except ValueError as e:
            raise ConfigError(str(e)) from None

    # ------------------------------------------------------------------ resolution
    def finalized(self, control_plane: bool = True):
        """The native options the exporter starts with: listen address parsed, host fallback,
        control-plane sockets checked / autodetected (``control_plane=False``: none)."""
        o = self._o.copy()
        if not control_plane:
            o.set("control_plane", "off")
        try:
            return o.finalized()
        except ValueError as e:
            raise ConfigError(str(e)) from None

    def validate(self) -> "Config":
        """The checks bin/gpumon-exporter runs before it starts (listen / debug addresses, the Influx
        push, the /metrics TLS files, the bearer token file). Raises ConfigError naming the problem."""
        err = self.finalized().validate()
        if err:
            raise ConfigError(err)
        return self

    @property
    def listen_addr(self) -> str:
        """Host part of ``listen`` ("" = every address, dual-stack)."""
        return parse_listen(self.listen)[0]

    @property
    def port(self) -> int:
        return parse_listen(self.listen)[1]

    def resolved_host(self) -> str:
        return self.finalized(control_plane=False).host


def parse_listen(listen: str):
    """``listen`` -> (host, port) by the native rule (csrc/core/http_server.cpp parse_listen)."""
    ok, host, port, err = core().parse_listen(str(listen))
    if not ok:
        raise ConfigError(err)
    return host, port


def redact_url(url: str) -> str:
    """``user:password@`` userinfo with the password masked (native redact_url)."""
    return core().redact_url(url)


def load_yaml(path: str) -> Dict[str, Any]:
    """A YAML file's ``gpumon:`` mapping read with PyYAML (tests compare it with the native parser)."""
    import yaml

    with open(path, "r", encoding="utf-8") as fh:
        data = yaml.safe_load(fh) or {}
    if not isinstance(data, dict):
        raise ValueError(f"{path}: top level must be a mapping")
    return data.get("gpumon", data)


_DEST = "cfgflag__"  # argparse dest prefix of the native flags


def add_cli_args(p: argparse.ArgumentParser) -> None:
    """The native flag table (csrc/core/options.cpp option_flags) on an argparse parser: the same
    vocabulary as bin/gpumon-exporter, each value checked by the native setters in from_args."""
    p.add_argument("--config", default=None, help="YAML config file (default $GPUMON_CONFIG)")
    p.add_argument("--compat", action="store_true",
                   help="reference behaviour: opt-in label mlgpu=mlgpu and 10 s interval")
    for f in core().option_flags():
        names = [f["flag"], *f["aliases"]]
        dest = _DEST + f["key"]
        if f["fixed"] is None:
            p.add_argument(*names, dest=dest, default=None, metavar=f["key"].upper(), help=f["help"])
        else:
            p.add_argument(*names, dest=dest, action="store_const", const=f["fixed"], default=None, help=f["help"])


def to_argv(ns: argparse.Namespace) -> List[str]:
    """The configuration flags of a parsed namespace, back as a command line for the native parser."""
    flags = core().option_flags()
    by_key = {}
    for f in flags:
        if f["fixed"] is None:
            by_key.setdefault(f["key"], f["flag"])
    fixed_only = {f["key"]: f["flag"] for f in flags if f["fixed"] is not None}
    argv = []
    if getattr(ns, "config", None):
        argv += ["--config", ns.config]
    if getattr(ns, "compat", False):
        argv.append("--compat")
    for k, v in vars(ns).items():
        if not k.startswith(_DEST) or v is None:
            continue
        key = k[len(_DEST):]
        if key in by_key:
            argv += [by_key[key], str(v)]
        else:  # a key only a fixed-value flag sets (--roctx, --influx-gzip, ...)
            argv.append(fixed_only[key])
    return argv


def from_args(ns: argparse.Namespace, env: Optional[Dict[str, str]] = None) -> Config:
    """defaults < file < environment < --compat < flags, by the native parser."""
    env = dict(os.environ if env is None else env)
    try:
        opts, _rest, warnings = core().Options.parse(to_argv(ns), env)
    except ValueError as e:
        raise ConfigError(str(e)) from None
    for w in warnings:
        logging.getLogger("gpumon").warning("%s", w)
    return Config(opts)
