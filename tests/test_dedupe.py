from gpumon.export import promtext


def test_duplicate_allocations_and_pids_are_single_series(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=1")
    a = {"pod_namespace": "ml", "pod_name": "jupyter-e-0", "container_name": "c", "gpu_index": 0}
    ex.set_allocations([a, dict(a)])
    ex.mock_set_procs([{"pid": 7, "device": 0, "vram_bytes": 1 << 30}, {"pid": 7, "device": 0, "vram_bytes": 1 << 30}])
    ex.tick()
    fam = promtext.parse(ex.metrics_text())  # raises on duplicate series
    assert promtext.one(fam, "pod_gpu_used_memory_bytes", pid="7") == 2 << 30
    assert len(promtext.values(fam, "pod_gpu_used_memory", pid="-")) == 1
