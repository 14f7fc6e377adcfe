#!/usr/bin/env python3
"""Generate deploy/grafana/gpumon-dashboard.json (Grafana 10 schema, Prometheus datasource).

Recreates the reference dashboards (described in SURVEY.md §2.5 from /root/reference/img/*.png)
in PromQL, then adds MI355X panels:
  * grafana.png              — per-card gauges "当前使用显存" (VRAM used) and "GPU使用率" (GPU util)
  * 2019 screenshot          — table "容器使用GPU情况", stats GPU总数 / 已占GPU数量 / 占GPU未开始使用 /
                               占GPU已使用完毕, time series "每个用户占用GPU的数量"
  * [new] per-XCD busy, xGMI per-link bandwidth, power/energy, temperatures, probe clocks,
          exporter self-metrics (sample + scrape latency p99).
"""

import json
import os

DS = {"type": "prometheus", "uid": "${datasource}"}
HOST = 'host=~"$host"'
_id = [0]


def panel(title, typ, targets, x, y, w, h, **kw):
    _id[0] += 1
    p = {"id": _id[0], "title": title, "type": typ, "datasource": DS,
         "gridPos": {"x": x, "y": y, "w": w, "h": h},
         "targets": [{"expr": e, "legendFormat": lf, "refId": chr(65 + i), "datasource": DS,
                      **({"format": "table", "instant": True} if typ == "table" else {})}
                     for i, (e, lf) in enumerate(targets)]}
    p.update(kw)
    return p


def build():
    panels = []
    y = 0
    # --- reference: allocation stat panels (2019 screenshot) ---
    stats = [("GPU总数 (GPUs total)", f'sum(gpumon_gpus{{{HOST},state="total"}})'),
             ("已占GPU数量 (allocated)", f'sum(gpumon_gpus{{{HOST},state="allocated"}})'),
             ("占GPU未开始使用 (allocated, idle)", f'sum(gpumon_gpus{{{HOST},state="allocated_idle"}})'),
             ("占GPU已使用完毕 (allocated, in use)", f'sum(gpumon_gpus{{{HOST},state="allocated_active"}})')]
    for i, (t, e) in enumerate(stats):
        panels.append(panel(t, "stat", [(e, "")], 6 * i, y, 6, 4))
    y += 4
    # --- reference: per-card gauges (grafana.png) ---
    panels.append(panel("当前使用显存 (VRAM used, MiB)", "gauge",
                        [(f'node_gpu_mem_used{{{HOST}}}', "{{host}} gpu{{gpu_id}}")], 0, y, 12, 7,
                        fieldConfig={"defaults": {"unit": "mbytes", "min": 0, "max": 294896}, "overrides": []}))
    panels.append(panel("GPU使用率 (GPU utilization %)", "gauge",
                        [(f'node_gpu_gpu_util{{{HOST}}}', "{{host}} gpu{{gpu_id}}")], 12, y, 12, 7,
                        fieldConfig={"defaults": {"unit": "percent", "min": 0, "max": 100}, "overrides": []}))
    y += 7
    # --- reference: container table + GPUs per user ---
    panels.append(panel("容器使用GPU情况 (GPU usage by container)", "table",
                        [(f'pod_gpu_used_memory{{{HOST}}}', ""), (f'pod_gpu_gpu_util{{{HOST}}}', "")], 0, y, 16, 9,
                        transformations=[{"id": "merge"}, {"id": "organize", "options": {
                            "excludeByName": {"Time": False, "__name__": True, "gpu_uuid": True},
                            "renameByName": {"Value #A": "used_memory", "Value #B": "gpu_util"},
                            "indexByName": {"Time": 0, "host": 1, "gpu_id": 2, "user_name": 3, "podname": 4,
                                            "containerid": 5, "pid": 6, "procressname": 7, "Value #B": 8,
                                            "Value #A": 9}}}]))
    panels.append(panel("每个用户占用GPU的数量 (GPUs held per user)", "timeseries",
                        [(f'count by (user_name) (pod_gpu_allocated{{{HOST}}})', "{{user_name}}")], 16, y, 8, 9))
    y += 9
    # --- MI355X extras ---
    panels.append(panel("Per-XCD GFX busy %", "heatmap",
                        [(f'gpu_xcd_busy_percent{{{HOST}}}', "{{host}} gpu{{gpu_id}} xcd{{xcd}}")], 0, y, 12, 8))
    panels.append(panel("xGMI per-link bandwidth (rx+tx)", "timeseries",
                        [(f'sum by (host, gpu_id, link) (gpu_xgmi_read_bytes_per_second{{{HOST}}} + '
                          f'gpu_xgmi_write_bytes_per_second{{{HOST}}})', "{{host}} gpu{{gpu_id}} link{{link}}")],
                        12, y, 12, 8, fieldConfig={"defaults": {"unit": "Bps"}, "overrides": []}))
    y += 8
    panels.append(panel("Socket power (W) / cap", "timeseries",
                        [(f'gpu_power_watts{{{HOST}}}', "{{host}} gpu{{gpu_id}}"),
                         (f'max(gpu_power_limit_watts{{{HOST}}})', "limit")], 0, y, 8, 8,
                        fieldConfig={"defaults": {"unit": "watt"}, "overrides": []}))
    panels.append(panel("Temperatures (°C)", "timeseries",
                        [(f'gpu_temperature_celsius{{{HOST}}}', "{{host}} gpu{{gpu_id}} {{sensor}}")], 8, y, 8, 8,
                        fieldConfig={"defaults": {"unit": "celsius"}, "overrides": []}))
    panels.append(panel("Throttle / violation %", "timeseries",
                        [(f'gpu_violation_percent{{{HOST}}}', "{{host}} gpu{{gpu_id}} {{kind}}")], 16, y, 8, 8))
    y += 8
    panels.append(panel("Energy rate (W, from accumulator)", "timeseries",
                        [(f'rate(gpu_energy_joules_total{{{HOST}}}[1m])', "{{host}} gpu{{gpu_id}}")], 0, y, 8, 8))
    panels.append(panel("HBM used (bytes)", "timeseries",
                        [(f'gpu_vram_used_bytes{{{HOST}}}', "{{host}} gpu{{gpu_id}}")], 8, y, 8, 8,
                        fieldConfig={"defaults": {"unit": "bytes"}, "overrides": []}))
    panels.append(panel("Memory controller activity %", "timeseries",
                        [(f'node_gpu_mem_bw_util{{{HOST}}}', "{{host}} gpu{{gpu_id}}")], 16, y, 8, 8))
    y += 8
    panels.append(panel("Probe: effective shader clock per XCD (MHz)", "timeseries",
                        [(f'gpu_probe_xcd_clock_mhz{{{HOST}}}', "{{host}} gpu{{gpu_id}} xcd{{xcd}}")], 0, y, 12, 8))
    panels.append(panel("PMC: MFMA utilisation % of wall time / KFD wave occupancy %", "timeseries",
                        [(f'gpu_mfma_util_percent{{{HOST}}}', "{{host}} gpu{{gpu_id}} mfma util"),
                         (f'gpu_cu_occupancy_percent{{{HOST}}}', "{{host}} gpu{{gpu_id}} wave slots held")], 12, y, 12, 8,
                        fieldConfig={"defaults": {"unit": "percent", "min": 0, "max": 100}, "overrides": []}))
    y += 8
    panels.append(panel("PMC: achieved MFMA TFLOP/s by operand type", "timeseries",
                        [(f'sum by (host, gpu_id, dtype) (gpu_mfma_tflops{{{HOST}}}) > 0',
                          "{{host}} gpu{{gpu_id}} {{dtype}}")], 0, y, 24, 8))
    y += 8
    panels.append(panel("Per-pod compute share (% of CUs holding the pod's waves)", "timeseries",
                        [(f'sum by (host, gpu_id, namespace, podname) (pod_gpu_proc_cu_occupancy_percent{{{HOST}}})',
                          "{{host}} gpu{{gpu_id}} {{namespace}}/{{podname}}")], 0, y, 12, 8,
                        fieldConfig={"defaults": {"unit": "percent", "min": 0, "max": 100}, "overrides": []}))
    panels.append(panel("XCD clock held below limit (% of time, by reason)", "timeseries",
                        [(f'avg by (host, gpu_id, reason) (gpu_xcd_clock_below_limit_percent{{{HOST},reason!="any"}})',
                          "{{host}} gpu{{gpu_id}} {{reason}}")], 12, y, 12, 8,
                        fieldConfig={"defaults": {"unit": "percent", "min": 0, "max": 100}, "overrides": []}))
    y += 8
    # Q4 fixed: the reference copied device utilisation onto every process row (gpu.py:205)
    panels.append(panel("Per-process GPU busy % (share of the interval with the process's waves resident)",
                        "timeseries",
                        [(f'max by (host, gpu_id, namespace, podname, pid) (pod_gpu_proc_gfx_util{{{HOST}}})',
                          "{{host}} gpu{{gpu_id}} {{namespace}}/{{podname}} pid {{pid}}")], 0, y, 12, 8,
                        fieldConfig={"defaults": {"unit": "percent", "min": 0, "max": 100}, "overrides": []}))
    panels.append(panel("Per-pod MFMA utilisation % (GPUs a pod uses alone; PMC)", "timeseries",
                        [(f'max by (host, gpu_id, namespace, podname) (pod_gpu_mfma_util_percent{{{HOST}}})',
                          "{{host}} gpu{{gpu_id}} {{namespace}}/{{podname}}")], 0, y + 8, 12, 8,
                        fieldConfig={"defaults": {"unit": "percent", "min": 0, "max": 100}, "overrides": []}))
    panels.append(panel("On-device samplers: PMC up / counter resets (tenant profilers)", "timeseries",
                        [(f'gpumon_pmc_up{{{HOST}}}', "{{host}} pmc up"),
                         (f'increase(gpumon_pmc_resets_total{{{HOST}}}[5m])', "{{host}} resets / 5m"),
                         (f'increase(gpumon_ondevice_helper_restarts_total{{{HOST}}}[1h])', "{{host}} helper restarts / 1h"),
                         (f'rate(gpumon_ondevice_helper_cpu_seconds_total{{{HOST}}}[5m])', "{{host}} helper CPU (cores)")],
                        12, y, 12, 8))
    # the reference dashboard titled node columns "(共享)" shared / "(独占)" exclusive by hand
    panels.append(panel("共享 / 独占: processes with waves resident per GPU (1 exclusive, >1 shared)", "timeseries",
                        [(f'gpu_active_processes{{{HOST}}}', "{{host}} gpu{{gpu_id}}")], 12, y + 8, 12, 8,
                        fieldConfig={"defaults": {"min": 0, "decimals": 0}, "overrides": []}))
    y += 16
    panels.append(panel("RAS: ECC errors by block (uncorrectable / correctable / deferred)", "table",
                        [(f'sum by (host, gpu_id, block, type) (gpu_ecc_errors_total{{{HOST}}}) > 0', "")], 0, y, 12, 8))
    panels.append(panel("RAS: retired HBM pages and poison / fatal events", "timeseries",
                        [(f'gpu_retired_pages{{{HOST}}}', "{{host}} gpu{{gpu_id}} retired pages"),
                         (f'gpu_ras_events_total{{{HOST}}} > 0', "{{host}} gpu{{gpu_id}} {{event}}")], 12, y, 12, 8))
    y += 8
    panels.append(panel("Exporter: /metrics p99 and tick p99 (s)", "timeseries",
                        [(f'histogram_quantile(0.99, sum by (le, host) (rate(gpumon_scrape_duration_seconds_bucket{{{HOST}}}[5m])))',
                          "{{host}} scrape p99"),
                         (f'histogram_quantile(0.99, sum by (le, host) (rate(gpumon_sample_duration_seconds_bucket{{{HOST}}}[5m])))',
                          "{{host}} tick p99")], 0, y, 12, 8,
                        fieldConfig={"defaults": {"unit": "s"}, "overrides": []}))
    panels.append(panel("Exporter: samples/s and errors", "timeseries",
                        [(f'rate(gpumon_samples_total{{{HOST}}}[1m])', "{{host}} samples/s"),
                         (f'sum by (host) (rate(gpumon_sample_errors_total{{{HOST}}}[5m]))', "{{host}} errors/s"),
                         (f'rate(gpumon_stale_samples_total{{{HOST}}}[1m])', "{{host}} stale (repeated table)/s")],
                        12, y, 12, 8))
    y += 8
    panels.append(panel("Firmware metrics table age (s); a frozen SMU table withholds rates", "timeseries",
                        [(f'gpu_metrics_table_age_seconds{{{HOST}}}', "{{host}} gpu{{gpu_id}} age"),
                         (f'gpu_metrics_table_frozen{{{HOST}}} > 0', "{{host}} gpu{{gpu_id}} FROZEN")], 0, y, 12, 8,
                        fieldConfig={"defaults": {"unit": "s"}, "overrides": []}))
    panels.append(panel("Exporter: HTTP loops at SCHED_FIFO / budget demotions / evictions (request floods)",
                        "timeseries",
                        [(f'gpumon_http_rt_loops{{{HOST}}}', "{{host}} RT loops"),
                         (f'rate(gpumon_http_rt_demotions_total{{{HOST}}}[5m])', "{{host}} demotions/s"),
                         (f'rate(gpumon_http_connections_evicted_total{{{HOST}}}[5m])', "{{host}} evicted conns/s")],
                        12, y, 12, 8))
    y += 8
    panels.append(panel("Exporter: failed process lists (last good list held up to 3 ticks)", "timeseries",
                        [(f'rate(gpumon_process_list_failures_total{{{HOST}}}[5m])', "{{host}} failed lists/s"),
                         (f'gpu_process_list_held{{{HOST}}} > 0', "{{host}} gpu{{gpu_id}} HELD"),
                         (f'rate(gpumon_occupancy_scan_failures_total{{{HOST}}}[5m])', "{{host}} KFD scan failures/s")],
                        0, y, 12, 8))
    # the reference's own transport: the InfluxDB push (where INFLUXDB_URL is set)
    panels.append(panel("InfluxDB compat push: up, pushes by result, seconds since the last success", "timeseries",
                        [(f'gpumon_influx_up{{{HOST}}}', "{{host}} up"),
                         (f'sum by (host, result) (rate(gpumon_influx_push_total{{{HOST}}}[5m]))', "{{host}} {{result}}/s"),
                         (f'time() - gpumon_influx_last_success_timestamp_seconds{{{HOST}}}', "{{host}} s since ok")],
                        12, y, 12, 8))
    y += 8
    panels.append(panel("Multi-GPU processes: peer contexts left out of pod_gpu rows (e.g. torchrun ranks opening every GPU)",
                        "timeseries",
                        [(f'gpumon_hidden_peer_gpu_contexts{{{HOST}}}', "{{host}} peer contexts"),
                         (f'gpumon_hidden_gpu_contexts{{{HOST}}}', "{{host}} empty contexts")], 0, y, 12, 6))
    # where /metrics is served over HTTPS (overlays/tls): certificate lifetime, rotations, refused handshakes
    panels.append(panel("/metrics over HTTPS: days left on the certificate, rotations, failed handshakes", "timeseries",
                        [(f'(gpumon_http_tls_cert_not_after_timestamp_seconds{{{HOST}}} - time()) / 86400', "{{host}} days left"),
                         (f'increase(gpumon_http_tls_reloads_total{{{HOST}}}[1h])', "{{host}} reloads {{result}} /h"),
                         (f'rate(gpumon_http_tls_handshake_failures_total{{{HOST}}}[5m])', "{{host}} failed handshakes/s")],
                        12, y, 12, 6))
    y += 6
    # the host link (interval rate from the firmware accumulator, profiles/r6_pcie_bandwidth.md) and the
    # hardware queues behind the peer-context rule (profiles/r6_kfd_queues.md)
    panels.append(panel("PCIe host link bandwidth (both directions, interval)", "timeseries",
                        [(f'gpu_pcie_bandwidth_bytes_per_second{{{HOST}}}', "{{host}} gpu{{gpu_id}}")], 0, y, 12, 8,
                        fieldConfig={"defaults": {"unit": "Bps"}, "overrides": []}))
    panels.append(panel("Hardware queues per process and GPU (0 = a context that never submitted work there)",
                        "timeseries",
                        [(f'max by (host, gpu_id, namespace, podname, pid) (pod_gpu_proc_queues{{{HOST}}})',
                          "{{host}} gpu{{gpu_id}} {{namespace}}/{{podname}} pid {{pid}}")], 12, y, 12, 8))
    return {
        "title": "gpumon — MI355X GPU cluster",
        "uid": "gpumon-mi355x",
        "schemaVersion": 39,
        "version": 1,
        "refresh": "5s",
        "time": {"from": "now-1h", "to": "now"},
        "tags": ["gpu", "amd", "mi355x", "kubernetes"],
        "templating": {"list": [
            {"name": "datasource", "type": "datasource", "query": "prometheus", "label": "Datasource"},
            {"name": "host", "type": "query", "datasource": DS, "label": "Node", "multi": True, "includeAll": True,
             "query": {"query": "label_values(node_gpu_gpu_util, host)", "refId": "hosts"}, "refresh": 2},
        ]},
        "panels": panels,
    }


if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gpumon-dashboard.json")
    with open(out, "w", encoding="utf-8") as fh:
        json.dump(build(), fh, ensure_ascii=False, indent=1)
    print(out)
