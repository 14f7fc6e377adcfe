"""One configuration implementation (csrc/core/options.cpp): bin/gpumon-exporter's command line and
the Python view (gpumon/config.py, `gpumon serve`) read the DaemonSet ConfigMap's YAML, GPUMON_<KEY>
env, the reference's NODE_NAME / INFLUXDB_URL and the flags through the same native table, so the
binary's --print-config and the Python view agree by construction (checked here end to end)."""

import json
import os
import subprocess

import pytest
import yaml

from gpumon.config import Config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin", "gpumon-exporter")
CLEAN_ENV = {k: v for k, v in os.environ.items() if not k.startswith("GPUMON_") and k not in ("NODE_NAME", "INFLUXDB_URL")}


def _print(*args, env=None):
    e = dict(CLEAN_ENV, **(env or {}))
    r = subprocess.run([BIN, *args, "--print-config"], capture_output=True, text=True, timeout=30, env=e)
    return r


def _py(path=None, env=None):
    cfg = Config()
    if path:
        cfg.apply_file(path)
    cfg.apply_env(dict(env or {}))
    return cfg.to_dict()


def _same(native, py):
    for k, v in native.items():
        if k == "host":
            continue
        assert k in py, k
        pv = py[k]
        if isinstance(v, float) or isinstance(pv, float):
            assert float(v) == pytest.approx(float(pv)), k
        else:
            assert v == pv, (k, v, pv)


def test_daemonset_configmap_parses_identically(tmp_path):
    (cm,) = [d for d in yaml.safe_load_all(open(os.path.join(ROOT, "deploy/k8s/gpumon-daemonset.yaml")))
             if d and d.get("kind") == "ConfigMap"]
    p = tmp_path / "config.yaml"
    p.write_text(cm["data"]["config.yaml"])
    r = _print("--config", str(p))
    assert r.returncode == 0, r.stderr
    _same(json.loads(r.stdout), _py(str(p)))


RICH = """\
# every value form the ConfigMap format allows
gpumon:
  interval: 0.1                 # 10 Hz
  listen: "127.0.0.1:9500"
  devices: [0, 2, 5]
  opt_in_label: 'mlgpu=mlgpu'
  user_regex: "^jupyter-([a-z]+)-"
  pod_label_allowlist:
    - team
    - app.kubernetes.io/name
  resource_names: [amd.com/gpu, "amd.com/gpu-cpx"]
  dra_drivers: []
  enable_pmc: yes
  enable_probe: true
  probe_every: 5
  pmc_counters: [SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, GRBM_COUNT]
  ras_every: 0
  gzip: off
  influx_url: http://influx:8086/write?db=k8s#not-a-comment
  control_plane: native
  not_a_key: 3                  # warned about, ignored
"""


def test_rich_file_env_and_flag_precedence(tmp_path):
    p = tmp_path / "rich.yaml"
    p.write_text(RICH)
    r = _print("--config", str(p))
    assert r.returncode == 0, r.stderr
    n = json.loads(r.stdout)
    _same(n, _py(str(p)))
    assert n["devices"] == ["0", "2", "5"] and n["dra_drivers"] == [] and n["gzip"] is False
    assert n["pod_label_allowlist"] == ["team", "app.kubernetes.io/name"]
    assert n["influx_url"] == "http://influx:8086/write?db=k8s#not-a-comment"
    assert "'not_a_key'" in r.stderr and "control_plane" not in r.stderr  # the ignored key is named
    # env over file, flags over env; the reference's env names
    env = {"GPUMON_INTERVAL": "2.5", "GPUMON_DEVICES": "1,3", "NODE_NAME": "gpu-node-7",
           "INFLUXDB_URL": "http://other/write", "GPUMON_FAKE_SOMETHING": "x"}
    r = _print("--config", str(p), "--interval", "0.5", env=env)
    assert r.returncode == 0, r.stderr
    n = json.loads(r.stdout)
    assert n["interval"] == 0.5 and n["devices"] == ["1", "3"] and n["host"] == "gpu-node-7"
    assert n["influx_url"] == "http://other/write"
    py = _py(str(p), env)
    assert py["devices"] == ["1", "3"] and py["influx_url"] == "http://other/write" and py["host"] == "gpu-node-7"


FLAG_SETS = [
    ["--procfs-root", "/host/proc", "--sysfs-root", "/host/sys", "--cri-socket", "/run/c.sock",
     "--pod-resources-socket", "/pr.sock", "--docker-socket", "/d.sock", "--pod-log-root", "/var/log",
     "--enable-pmc", "--enable-probe-kernel", "--device-timeout", "3.5", "--http-threads", "3"],
    ["--procfs", "/host/proc", "--sysfs", "/host/sys", "--cri", "/run/c.sock", "--pod-resources", "/pr.sock",
     "--docker", "/d.sock", "--pod-logs", "/var/log", "--pmc", "--probe", "--ras-every", "7", "--ras-slices", "2",
     "--dra-drivers", "none", "--pmc-mode", "window", "--probe-every", "4"],
    ["--no-cri", "--no-pod-resources", "--compat"],
    ["--compat", "--interval", "1", "--opt-in-label", "team=ml"],
    ["--control-plane", "off"],
]


@pytest.mark.parametrize("flags", FLAG_SETS, ids=["python-spellings", "native-spellings", "off-switches", "compat",
                                                   "control-plane-off"])
def test_both_entry_points_take_each_others_flags(flags):
    """One flag vocabulary: a command line written for `gpumon serve` runs the image's native
    entrypoint unchanged and the other way round, with the same resulting configuration."""
    import argparse

    from gpumon.config import add_cli_args, from_args

    r = _print(*flags)
    assert r.returncode == 0, r.stderr
    native = json.loads(r.stdout)
    ap = argparse.ArgumentParser()
    add_cli_args(ap)
    cfg = from_args(ap.parse_args(flags), env={})
    _same(native, cfg.to_dict())
    if "--control-plane" in flags:
        # off: every metadata source of the finalized options is cleared
        assert native["control_plane"] == "off"
        assert all(v == "" for v in cfg.finalized().exporter_sources.values())


@pytest.mark.parametrize("args,rc,want", [
    (["--help"], 0, "usage: gpumon-exporter"),
    (["--no-such-flag"], 2, "unknown flag --no-such-flag"),
    (["--interval"], 2, "usage: gpumon-exporter"),  # a flag missing its value
    (["--control-plane", "maybe"], 2, "--control-plane: native or off, not 'maybe'"),
    (["--interval", "fast"], 2, "interval"),
    (["--listen", "[::1"], 2, "listen"),
    (["--config"], 2, "--config: missing value"),
    (["--config="], 2, "--config: missing value"),
])
def test_native_binary_refuses_bad_command_lines(args, rc, want):
    r = subprocess.run([BIN, *args], capture_output=True, text=True, timeout=30, env=CLEAN_ENV)
    assert r.returncode == rc, (r.returncode, r.stderr[-1000:])
    assert want in r.stderr, r.stderr[-1000:]


def test_config_env_var_names_the_file(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("gpumon:\n  ras_every: 7\n")
    r = _print(env={"GPUMON_CONFIG": str(p)})
    assert r.returncode == 0 and json.loads(r.stdout)["ras_every"] == 7


@pytest.mark.parametrize("text,msg", [
    ("gpumon:\n  interval: fast\n", "interval: not a number"),
    ("gpumon:\n  probe_every: 1.5\n", "probe_every: not an integer"),
    ("gpumon:\n  gzip: maybe\n", "gzip: not a boolean"),
    ("gpumon:\n  rates:\n    xgmi: 1\n", "line 3: nested mappings"),
    ("gpumon:\n  interval: 1\n  interval: 2\n", "line 3: duplicate key"),
    ("gpumon:\n  devices: [0, 1\n", "line 2: unterminated flow list"),
    ("gpumon:\n  user_regex: \"abc\n", "unterminated"),
    ("gpumon:\n  listen: {a: b}\n", "unsupported YAML construct"),
    ("gpumon:\n  devices: [[0], 1]\n", "line 2: nested collections are not supported"),
    ("gpumon:\n  devices: [\"0, 1]\n", "line 2: unterminated quoted value"),
    ("gpumon:\n\tinterval: 2\n", "line 2: tab indentation"),
    ("other: 1\n", None),  # no gpumon: mapping: flat file, unknown key -> warning only
])
def test_bad_files_fail_with_the_line(tmp_path, text, msg):
    p = tmp_path / "bad.yaml"
    p.write_text(text)
    r = _print("--config", str(p))
    if msg is None:
        assert r.returncode == 0 and "'other'" in r.stderr
    else:
        assert r.returncode == 2 and msg in r.stderr, r.stderr


def test_bad_env_value_is_fatal():
    r = _print(env={"GPUMON_INTERVAL": "soon"})
    assert r.returncode == 2 and "GPUMON_INTERVAL" in r.stderr


def test_binary_serves_with_the_configmap(tmp_path):
    """--once with a config file drives the sampler (mock backend from the file)."""
    p = tmp_path / "c.yaml"
    p.write_text("gpumon:\n  backend: 'mock:gpus=3'\n  pod_resources_socket: ''\n  cri_socket: none\n"
                 "  host: from-file\n")
    r = subprocess.run([BIN, "--config", str(p), "--once"], capture_output=True, text=True, timeout=60,
                       env=CLEAN_ENV)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count('node_gpu_gpu_util{host="from-file"') == 3


# ---------------------------------------------------------------- parser vs PyYAML (property-based)
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

_word = st.text(alphabet="abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_./-:=@ ", min_size=1,
                max_size=20).filter(lambda s: s.strip() == s)
_scalar = st.one_of(_word, st.integers(-10 ** 6, 10 ** 6), st.booleans(),
                    st.floats(-1e6, 1e6, allow_nan=False).map(lambda f: round(f, 3)))
_value = st.one_of(_scalar, st.lists(st.one_of(_word, st.integers(0, 999)), max_size=5))
# keys PyYAML (YAML 1.1) would resolve to a bool / null are not config keys: leave them out
_YAML11_KEYWORDS = {"y", "n", "yes", "no", "on", "off", "true", "false", "null"}
_doc = st.dictionaries(st.from_regex(r"[a-z][a-z0-9_]{0,11}", fullmatch=True).filter(lambda k: k not in _YAML11_KEYWORDS),
                       _value, max_size=8)


def _as_text(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def _dump_scalar(v):
    t = yaml.safe_dump(v, width=10 ** 6)
    return t[:-len("\n...\n")] if t.endswith("\n...\n") else t.rstrip("\n")


def _dump(doc, flow_lists, wrap):
    """Block mapping (the ConfigMap's shape) with lists in flow or block style, scalars exactly as
    PyYAML would emit them (quoting included)."""
    ind = "  " if wrap else ""
    out = ["gpumon:"] if wrap else []
    for k, v in doc.items():
        if isinstance(v, list) and (flow_lists or not v):
            out.append(f"{ind}{k}: " + yaml.safe_dump(v, default_flow_style=True, width=10 ** 6).strip())
        elif isinstance(v, list):
            out.append(f"{ind}{k}:")
            out.extend(f"{ind}  - {_dump_scalar(x)}" for x in v)
        else:
            out.append(f"{ind}{k}: {_dump_scalar(v)}")
    return "\n".join(out) + "\n"


@settings(max_examples=300, deadline=None)
@given(doc=_doc.filter(bool), flow=st.booleans(), wrap=st.booleans())
def test_yaml_subset_agrees_with_pyyaml(doc, flow, wrap):
    from gpumon import core

    body = _dump(doc, flow, wrap)
    got = core().parse_yaml_subset(body)
    want = yaml.safe_load(body)
    want = want.get("gpumon", want) if wrap else want
    assert list(got) == list(want)
    for k, v in want.items():
        exp = [_as_text(x) for x in v] if isinstance(v, list) else [_as_text(v)]
        g = got[k]
        if isinstance(v, float):
            assert float(g[0]) == pytest.approx(v)
        else:
            assert g == exp, (k, g, exp, body)


def test_metric_filter_keys_parse_identically(tmp_path):
    """metrics_include / metrics_exclude: YAML block list, env, and the binary's flag."""
    p = tmp_path / "filter.yaml"
    p.write_text("gpumon:\n  metrics_exclude:\n    - 'gpu_xcd_*'\n    - gpu_probe_*\n  metrics_include: [node_gpu_*, 'gpu_*']\n")
    r = _print("--config", str(p))
    assert r.returncode == 0, r.stderr
    n = json.loads(r.stdout)
    assert n["metrics_exclude"] == ["gpu_xcd_*", "gpu_probe_*"] and n["metrics_include"] == ["node_gpu_*", "gpu_*"]
    _same(n, _py(str(p)))
    env = {"GPUMON_METRICS_EXCLUDE": "pod_gpu_*,gpumon_*"}
    n = json.loads(_print("--config", str(p), env=env).stdout)
    assert n["metrics_exclude"] == ["pod_gpu_*", "gpumon_*"] == _py(str(p), env)["metrics_exclude"]
    n = json.loads(_print("--metrics-exclude", "gpu_xcd_*").stdout)
    assert n["metrics_exclude"] == ["gpu_xcd_*"] and n["metrics_include"] == []


def test_environment_only_knobs_are_documented():
    """Every GPUMON_* variable the native code reads with getenv() (the test fakes' GPUMON_FAKE_*
    aside) is in docs/configuration.md's environment-only table, and the table lists no other."""
    import re
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_config_doc

    read = set()
    for base, _, files in os.walk(os.path.join(ROOT, "csrc")):
        for f in files:
            if f.endswith((".cpp", ".h", ".hip")):
                text = open(os.path.join(base, f)).read()
                read |= set(re.findall(r'getenv\("(GPUMON_[A-Z0-9_]+)"\)', text))
                read |= set(re.findall(r'"(GPUMON_[A-Z0-9_]+)="', text))  # read from an envp block
    read = {v for v in read if not v.startswith("GPUMON_FAKE_")}
    listed = {name for name, *_ in gen_config_doc.ENV_ONLY}
    assert read == listed, (read - listed, listed - read)
    doc = open(os.path.join(ROOT, "docs", "configuration.md")).read()
    assert doc == gen_config_doc.render(), "docs/configuration.md is stale: python tools/gen_config_doc.py"


def test_drifts_of_round_5_are_gone(monkeypatch, tmp_path):
    """the two parsers disagreed on the CRI autodetect list (Python tried
    /var/run/containerd/containerd.sock, native did not) and on the host fallback (Python NODE_NAME
    -> host name -> no_name, native NODE_NAME -> no_name). Both now come from options.cpp."""
    import socket

    from gpumon import core

    socks = core().cri_autodetect_sockets()
    assert "/var/run/containerd/containerd.sock" in socks and socks[0] == "/run/containerd/containerd.sock"
    monkeypatch.delenv("NODE_NAME", raising=False)
    want = socket.gethostname() or "no_name"
    assert Config().resolved_host() == want
    p = tmp_path / "c.yaml"
    p.write_text("gpumon:\n  backend: 'mock:gpus=1'\n  control_plane: 'off'\n")
    r = subprocess.run([BIN, "--config", str(p), "--once"], capture_output=True, text=True, timeout=60, env=CLEAN_ENV)
    assert r.returncode == 0, r.stderr
    assert f'node_gpu_gpu_util{{host="{want}"' in r.stdout


def test_python_view_has_no_key_table_of_its_own():
    """No key, default or autodetect list in two languages: gpumon/config.py names none of them."""
    import re

    src = open(os.path.join(ROOT, "gpumon", "config.py")).read()
    assert "containerd" not in src and "turing-gpu-notebook" not in src and "9400" not in src
    assert "@dataclass" not in src and not re.search(r"^    \w+: (str|int|float|bool|List)\b.* = ", src, re.M)
    from gpumon import core

    keys = {k["key"] for k in core().option_keys()}
    assert {"interval", "listen", "host", "control_plane", "cri_socket", "debug_listen", "pcie_bw_unit_bytes"} <= keys


def test_env_only_list_is_the_docs_list(core):
    """The runtime's own list of environment-only variables (what a typo is checked against) is the
    documented one, which test_environment_only_knobs_are_documented ties to the getenv() calls."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_config_doc

    assert sorted(core.env_only_variables()) == sorted(name for name, *_ in gen_config_doc.ENV_ONLY)


def test_misspelt_gpumon_variable_is_named(caplog):
    """GPUMON_INTERVALL=5 is not a key: both entry points say so and go on with the default; real
    keys, environment-only variables and the test fakes' GPUMON_FAKE_* pass silently."""
    env = {"GPUMON_INTERVALL": "5", "GPUMON_INTERVAL": "2", "GPUMON_HTTP_SNDBUF": "0", "GPUMON_FAKE_PCI": "x",
           # Kubernetes service links of a Service named gpumon (enableServiceLinks left on)
           "GPUMON_SERVICE_HOST": "10.0.0.1", "GPUMON_PORT": "tcp://10.0.0.1:9400",
           "GPUMON_PORT_9400_TCP_ADDR": "10.0.0.1"}
    r = _print(env=env)
    assert r.returncode == 0 and json.loads(r.stdout)["interval"] == 2.0
    assert "GPUMON_INTERVALL is neither a configuration key" in r.stderr
    assert "GPUMON_HTTP_SNDBUF" not in r.stderr and "GPUMON_FAKE_PCI" not in r.stderr
    assert "SERVICE_HOST" not in r.stderr and "GPUMON_PORT" not in r.stderr
    import logging

    with caplog.at_level(logging.WARNING, logger="gpumon"):
        assert Config().apply_env(env).interval == 2.0
    assert [m for m in caplog.messages if "GPUMON_INTERVALL" in m] and not [m for m in caplog.messages
                                                                          if "SNDBUF" in m]


def test_inline_flag_values_escapes_and_retired_keys(tmp_path):
    """`--flag=value` as well as `--flag value`; a fixed-value flag refuses a value; YAML double-quote
    escapes (\\n, \\t, \\") in scalars and flow lists; influx_token from the file (redacted on print);
    the retired `ondevice` key is accepted without effect; a missing file is named."""
    r = _print("--interval=2.5", "--listen=127.0.0.1:9500")
    n = json.loads(r.stdout)
    assert r.returncode == 0 and n["interval"] == 2.5 and n["listen"] == "127.0.0.1:9500"
    r = _print("--influx-extended=false")
    assert r.returncode == 2 and "--influx-extended takes no value" in r.stderr
    p = tmp_path / "c.yaml"
    p.write_text('gpumon:\n  user_regex: "a\\tb\\nc"\n  metrics_exclude: ["x\\"y", z]\n'
                 '  influx_token: "s3cret"\n  ondevice: true\n')
    r = _print("--config", str(p))
    assert r.returncode == 0, r.stderr
    n = json.loads(r.stdout)
    assert n["user_regex"] == "a\tb\nc" and n["metrics_exclude"] == ['x"y', "z"]
    assert n["influx_token"] == "***" and "s3cret" not in r.stdout and "ondevice" not in r.stderr
    r = _print("--config", str(tmp_path / "missing.yaml"))
    assert r.returncode == 2 and "cannot read" in r.stderr and "missing.yaml" in r.stderr
