"""gpumon — MI355X-native Kubernetes GPU telemetry exporter.

Capabilities of the reference agent (/root/reference/gpu.py: node_gpu + pod_gpu measurements,
DaemonSet deployment, NODE_NAME / INFLUXDB_URL configuration) re-designed for AMD Instinct MI355X:

* ``gpumon._core``  — C++ core (libamd_smi via dlopen, sampler, /proc attribution, Prometheus +
  Influx renderers, epoll HTTP server).  Built in-tree by ``make`` / ``__graft_entry__.build()``.
* ``gpumon._hip``   — hand-written gfx950 HIP kernels: on-device probe (per-XCD clock, dispatch
  latency, pinned ring buffer) and synthetic MFMA / HBM load generators.
  The core also holds the k8s control plane: CRI + kubelet PodResources (+ opt-in Docker) pollers
  for pod / namespace / user labels and allocated-but-idle GPUs (csrc/core/grpc_lite.cpp).
* ``gpumon.monitor`` / ``gpumon.cli`` — config, ``gpumon serve|once|top|doctor|...``.
* ``gpumon.parallel`` — RCCL/xGMI load generators used to validate the per-link xGMI counters.
"""

__version__ = "0.1.0"

from ._native import core, hip, native_available  # noqa: F401
