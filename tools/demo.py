"""Mock 8-GPU node + fake kubelet / CRI: the full pod_gpu path (pod, namespace, user labels and an
allocated-but-idle row) without a cluster or a GPU. The fake kubelet is a test oracle
(tests/oracles/attribution/fake_kubelet.py, needs grpcio) and is not shipped in the image, so the
demo lives here rather than in `gpumon`'s CLI.

    python tools/demo.py [--gpus 8] [--listen 127.0.0.1:9400] [--seconds 0]
    curl -s 127.0.0.1:9400/metrics | grep pod_gpu_used_memory
"""

import argparse
import os
import signal
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main() -> int:
    from gpumon.config import Config
    from gpumon.monitor import GpuMonitor
    from oracles.attribution.fake_kubelet import FakeKubelet, FakePod

    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--listen", default="127.0.0.1:9400")
    ap.add_argument("--interval", type=float, default=1.0)
    ap.add_argument("--seconds", type=float, default=0, help="stop after this long (0 = until Ctrl-C)")
    args = ap.parse_args()

    d = tempfile.mkdtemp(prefix="gpumon-demo-")
    k = FakeKubelet(podres_socket=f"{d}/kubelet.sock", cri_socket=f"{d}/cri.sock").start()
    cid = "%064x" % 0xC0FFEE
    k.pods = [FakePod("turing-gpu-notebook-alice-5d8f-x1", "ml", "uid-alice", labels={"mlgpu": "mlgpu"},
                      containers={"notebook": (cid, ["0000:05:00.0"])}),
              FakePod("jupyter-q-0", "research", "uid-q", containers={"main": ("%064x" % 0xBEEF, ["0000:25:00.0"])})]
    cfg = Config(backend=f"mock:gpus={args.gpus}", listen=args.listen, interval=args.interval,
                 cri_socket=k.cri_socket, pod_resources_socket=k.podres_socket, metadata_refresh=2.0)
    mon = GpuMonitor(cfg).start()
    mon.ex.mock_set_procs([{"pid": os.getpid(), "device": 0, "name": "python train.py", "vram_bytes": 12 << 30}])
    print(f"demo exporter at {mon.url} (fake kubelet in {d}); Ctrl-C to stop", flush=True)
    stop = threading.Event()
    for s in (signal.SIGINT, signal.SIGTERM):
        signal.signal(s, lambda *_: stop.set())
    end = time.time() + args.seconds if args.seconds > 0 else float("inf")
    while not stop.wait(0.5) and time.time() < end:
        pass
    mon.stop()
    k.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
