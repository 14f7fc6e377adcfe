"""bench.py driver contract on CPU: single process and 2-rank torch.distributed (gloo).

The driver runs `python bench.py --gpus N --steps K --warmup W` (N=1) and, for N>1,
`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py`; rank 0
prints exactly one JSON line with the BASELINE metric name.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check_exporter(d, world):
    """the line measures the SHIPPED binary, run as its own process, attributing
    the bench's load as a foreign tenant; and it carries what the first 8-GPU record must settle."""
    info = d["exporter_info"]
    assert d["exporter"] == "bin/gpumon-exporter" and info["mode"] == "child"
    assert d["exporter_pid"] == info["pid"] and d["exporter_pid"] not in info["tenant_pids"]
    assert info["spawned_before_hip"] is True and not info["exporter_pid_in_rows"]
    assert len(info["tenant_pids"]) == world and info["rss_mb"] > 0
    # the child's CPU per thread name (all of that process is the exporter)
    thr = d["exporter_thread_cpu_millicores"]
    assert {"gpumon-sampler", "gpumon-http"} <= set(thr) and d["exporter_cpu_millicores"] == pytest.approx(
        sum(thr.values()), abs=0.05)
    # per sampled device: its own calls' time per tick
    assert [x["gpu"] for x in d["per_device_tick_ms"]] == list(range(d["sampled_devices"]))
    assert all(x["t_device_mean_ms"] > 0 and "t_procs_mean_ms" in x for x in d["per_device_tick_ms"])
    # the process group's world size as every rank saw it
    assert sorted(x["rank"] for x in d["ranks"]) == list(range(world))
    assert all(x["world_size"] == world for x in d["ranks"])


def _check(d, n, steps, warmup):
    assert REQUIRED <= set(d)
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    assert set(d["config"]) >= {"model", "global_batch", "seq_len", "parallelism"}
    assert d["value"] > 0 and d["scrape_p99_ms"] > 0 and d["scrape_errors"] == 0
    # K waited-for ticks; at a 0.1 s interval the closing barrier (CPU all-reduces) can span another
    assert steps <= d["ticks"] <= steps + 2


@pytest.mark.parametrize("dist", [False, True], ids=["plain", "dist"])
def test_bench_single_process(dist):
    """`--dist`: the torchrun code path (process group, barriers, MAX over ranks) with one rank."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(29600 + os.getpid() % 1000))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--interval", "0.1", "--idle-s", "1"] + (["--dist"] if dist else []),
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    _check(lines[0], 1, 3, 1)
    _check_exporter(lines[0], 1)
    assert lines[0]["value"] == pytest.approx(10.0, rel=0.2)  # 1 device x 10 Hz
    idle = lines[0]["scrape_idle"]  # untimed idle reference before the load
    assert idle["scrapes"] > 5 and idle["scrape_errors"] == 0 and idle["scrape_p99_ms"] > 0 and idle["ticks"] >= 5
    d = lines[0]
    # tail statistics worth quoting -- p99.9, the exporter's own service time of the
    # same requests (exact, server side), and what `value` measures
    assert d["scrape_p999_ms"] >= d["scrape_p99_ms"] > 0 and d["scrape_rate_hz"] >= 100
    # the server stamps a scrape's end after its write returns: a thread preempted right there (a
    # busy CPU box) logs a little more than the client saw, so the bound carries a 5 ms allowance
    assert d["server_scrapes"] == d["scrapes"] and 0 < d["server_scrape_p99_ms"] <= d["scrape_max_ms"] + 5.0
    assert "interval" in d["value_note"]
    assert idle["server_scrape_p99_ms"] > 0 and idle["scrape_p999_ms"] >= idle["scrape_p99_ms"]
    # sampler capacity: a 1 ms-interval exporter after the timed region goes far past 1/interval
    cap = d["capacity"]
    assert "error" not in cap, cap
    assert cap["interval_ms"] == 1.0 and cap["ticks_logged"] > 0 and cap["samples_per_sec_per_gpu"] > 100
    assert [x["gpu"] for x in d["per_gpu_rows"]] == [0] and d["per_gpu_rows"][0]["active_processes"] is not None
    assert "hidden_contexts" in d and "hidden_peer_contexts" in d and "rows_per_user" in d
    assert isinstance(d["hidden_context_detail"], list) and isinstance(d["hidden_context_reasons"], dict)
    hl = d["host_load"]
    assert hl["cpus_usable"] >= 1 and hl["loadavg_1m_before"] is not None and hl["loadavg_1m_after"] >= 0


@pytest.mark.slow
def test_bench_two_ranks_gloo():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(29600 + os.getpid() % 300),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--interval", "0.1", "--allreduce-mb", "1", "--idle-s", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    _check(lines[0], 2, 3, 1)
    assert "all-reduce" in lines[0]["config"]["parallelism"]
    x = lines[0]["xgmi"]
    assert x["allreduce_mb"] == 1
    # 2 ranks: a ring all-reduce moves (2(n-1)/n) * S = 1 MiB out of each rank per step
    assert x["expected_tx_GBps_per_gpu"] > 0
    assert "exporter_tx_GBps_per_gpu" in x and "exporter_vs_expected" in x
    # the timed region starts on a tick and each step's all-reduces run inside its interval: K
    # steps span K intervals, so the whole-node rate is N / interval (was ~0.9x with the last
    # step's reductions past the last tick and a random start phase)
    assert lines[0]["value"] == pytest.approx(2 / 0.1, rel=0.12)


def test_bench_runs_without_torch():
    """A lean image (the exporter's plus the tools) has no PyTorch: the single-process bench still
    runs, on the native HIP path for the GPU check and loads."""
    code = ("import sys, runpy; sys.modules['torch'] = None; sys.argv = ['bench.py', '--steps', '2', '--warmup', '1', "
            "'--interval', '0.1', '--idle-s', '0.5']; runpy.run_path('bench.py', run_name='__main__')")
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    _check(line, 1, 2, 1)


def test_value_counts_fresh_samples_only():
    """`value` is fresh device samples/s. A mock SMU refreshing at 50 Hz sampled
    every 5 ms repeats most tables: value stays near 50 per GPU while the exporter took ~200 samples/s,
    and both counts are in the line."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "200", "--warmup", "2",
                        "--interval", "0.005", "--idle-s", "0", "--capacity-s", "0", "--scrape-rate", "50",
                        "--backend", "mock:gpus=1,mode=load,firmware_hz=50"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (d,) = _json_lines(r.stdout)
    assert d["value"] <= 50 * 1.15, d["value"]
    # ~4 samples per fresh table at 5 ms / 50 Hz; 2 leaves room for a loaded CI host
    assert d["samples_total"] >= 2 * d["value"] * d["ms_per_step"] * d["steps"] / 1e3
    assert d["stale_samples"] == d["samples_total"] - round(d["value"] * d["ms_per_step"] * d["steps"] / 1e3)
    assert d["devices"] == [{"hip_ordinal": 0, "bdf": "0000:05:00.0", "gpu_id": "0"}]
    assert d["device_check"]["ok"]


@pytest.mark.slow
def test_bench_eight_ranks_exact_scale_command():
    """the driver's SCALE command shape at N=8 (torchrun, one rank per GPU, no extra
    flags) over gloo + the mock backend: one line from rank 0 with 8 sampled devices, each HIP
    ordinal paired with a distinct device, and the whole-node rate N / interval."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(29000 + os.getpid() % 400),
                        os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    _check(d, 8, 3, 1)
    _check_exporter(d, 8)
    assert d["sampled_devices"] == 8 and d["config"]["interval_s"] == 1.0
    assert [x["hip_ordinal"] for x in d["devices"]] == list(range(8))
    assert len({x["gpu_id"] for x in d["devices"]}) == 8 and d["device_check"]["ok"]
    # per-GPU row accounting in the SCALE record (one load process per rank here,
    # each on its own GPU: one row per GPU, no peer context on the mock)
    assert [x["gpu"] for x in d["per_gpu_rows"]] == list(range(8))
    assert all(set(x) >= {"rows", "pids", "idle_rows", "active_processes"} for x in d["per_gpu_rows"])
    assert d["hidden_peer_contexts"] == 0 and isinstance(d["rows_per_user"], dict)
    # 8 ranks' 256 MB gloo all-reduces share the builder's CPUs with the exporter: the last step's
    # reductions can run past its tick, so the whole-node rate is N / interval within 25 % here,
    # with the rest of the parallel CPU suite on the same CPUs (exact on the GPU node, where RCCL
    # moves the bytes)
    assert d["value"] == pytest.approx(8.0, rel=0.25)


def test_inprocess_exporter_is_the_ab_mode():
    """--exporter inprocess keeps the old embedding (the same core through the bindings) for A/B."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--exporter", "inprocess", "--steps", "3",
                        "--warmup", "1", "--interval", "0.1", "--idle-s", "0.5", "--capacity-s", "0"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (d,) = _json_lines(r.stdout)
    _check(d, 1, 3, 1)
    assert d["exporter"] == "in-process (gpumon._core)" and d["exporter_pid"] == d["exporter_info"]["tenant_pids"][0]
    assert set(d["exporter_thread_cpu_millicores"]) <= {"gpumon-sampler", "gpumon-http", "gpumon-dev0", "gpumon-proc0"}


def test_child_exporter_uses_the_daemonset_config(tmp_path):
    """The child reads a config file with the DaemonSet ConfigMap's keys plus the bench's overrides;
    its /debug views answer on loopback only."""
    from gpumon.export.child import ChildExporter, daemonset_config

    base = daemonset_config()
    assert base["interval"] == 1.0 and base["listen"] == ":9400" and "pod_resources_socket" in base
    ex = ChildExporter(dict(base, backend="mock:gpus=2", interval=0.1, log_level="warn"), str(tmp_path)).start()
    try:
        assert ex.wait_ticks(2, 10)
        st = ex.state()
        assert st["pid"] == ex.pid != os.getpid() and len(st["statics"]) == 2
        text = (tmp_path / "gpumon-config.yaml").read_text()
        assert "debug_listen: \"127.0.0.1:" in text and "user_prefix: \"turing-gpu-notebook-\"" in text
        ticks = ex.ticks(0)
        assert ticks and all(len(t["dev"]) == 2 for t in ticks)
        assert "node_gpu_gpu_util" in ex.metrics()
    finally:
        assert ex.stop() == 0


def test_post_measurement_extras_are_time_bounded():
    """The link map and the capacity run happen after the timed region and before the line is
    printed: a stuck one is given up on (and an error recorded) instead of holding the line back."""
    import importlib.util
    import time

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    t0 = time.monotonic()
    r = bench._bounded(time.sleep, 0.3, 30)
    assert r == {"error": "timed out after 0.3 s"} and time.monotonic() - t0 < 2
    assert bench._bounded(lambda: 1 / 0, 5) == {"error": "ZeroDivisionError: division by zero"}
    assert bench._bounded(lambda x: {"ok": x}, 5, 7) == {"ok": 7}


@pytest.mark.slow
def test_ranks_sharing_a_gpu_rehearsal():
    """--ranks-per-gpu K: the torchrun path with K ranks on each GPU (a 1-GPU box rehearsing the
    multi-rank record: every rank's tenant row on the shared GPU, the world size each rank saw).
    The process group is gloo (RCCL takes one rank per GPU) and the line says it is a rehearsal."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(28600 + os.getpid() % 300),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--ranks-per-gpu", "2", "--steps", "3",
                        "--warmup", "1", "--interval", "0.1", "--idle-s", "0.5", "--capacity-s", "0"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    (d,) = _json_lines(r.stdout)
    _check(d, 1, 3, 1)
    _check_exporter(d, 2)
    assert d["sampled_devices"] == 1 and "2 ranks per GPU (rehearsal)" in d["config"]["parallelism"]
    assert d["xgmi"] is None and [x["device"] for x in sorted(d["ranks"], key=lambda x: x["rank"])] == [0, 0]
    assert all(x["backend"] == "gloo" for x in d["ranks"]) and "wall time" in d["load_rates"]
    assert d["value"] == pytest.approx(1 / 0.1, rel=0.2)


def test_ranks_per_gpu_must_divide_the_world():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--ranks-per-gpu", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "does not divide the world size 3" in r.stderr


def test_child_config_file_round_trips_through_the_native_parser(tmp_path):
    """write_config's scalars are what the binary reads back: quotes, backslashes, a tab, non-ASCII
    text (the reference's Chinese dashboard titles are the kind of value a label may carry)."""
    from gpumon.export.child import BINARY, write_config

    want = {"user_prefix": 'notebook-"q"\\\t用户-', "metrics_exclude": ["a,b", "gpu_xcd_*"], "interval": 0.5,
            "gzip": False}
    p = tmp_path / "c.yaml"
    write_config(want, str(p))
    env = {k: v for k, v in os.environ.items() if not k.startswith("GPUMON_")}
    r = subprocess.run([BINARY, "--config", str(p), "--print-config"], capture_output=True, text=True, timeout=30,
                       env=env)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout)
    assert {k: got[k] for k in want} == want


def test_scale_report_reads_bench_lines(tmp_path):
    """tools/scale_report.py turns per-N bench lines into the 8-GPU table and names what is off:
    rows per GPU against ranks per GPU, world sizes, scaling efficiency."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scale_report

    def line(n, value, rows, ws):
        return {"metric": "m", "n_gpus": n, "value": value, "scrape_p99_ms": 0.1, "server_scrape_p99_ms": 0.02,
                "tick_mean_ms": 0.3, "tick_p99_ms": 0.5, "overruns": 0, "exporter_cpu_millicores": 7.0 * n,
                "per_device_tick_ms": [{"gpu": g, "t_device_mean_ms": 0.1 + 0.01 * g} for g in range(n)],
                "per_gpu_rows": [{"gpu": g, "rows": rows} for g in range(n)],
                "ranks": [{"rank": r, "world_size": ws} for r in range(n if n > 1 else 1)],
                "hidden_context_reasons": {"peer": n * (n - 1)} if n > 1 else {},
                "xgmi": {"exporter_vs_expected": 0.98, "link_map": {"peers_matched": n - 1, "peers": n - 1,
                                                                     "rates_within_15pct": n - 1}} if n > 1 else None,
                "device_check": {"ok": True}}

    p = tmp_path / "scale.json"
    p.write_text(json.dumps({"runs": [line(1, 1.0, 1, 1), line(2, 2.0, 1, 2), line(8, 7.2, 8, 8)]}))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scale_report.py"), str(p)], capture_output=True,
                       text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert "| 8 | 7.2000 | 0.9000 | 0.900 |" in out and "0.100-0.170" in out and "7/7 peers" in out
    assert "N=8: workload rows per GPU [8, 8, 8, 8, 8, 8, 8, 8] differ from ranks per GPU (1)" in out
    assert "N=8: scaling efficiency 0.900 < 0.95" in out and "N=2" not in out.split("\n\n")[-1]
    assert [x["n"] for x in scale_report.rows(scale_report._lines(str(p)))] == [1, 2, 8]
