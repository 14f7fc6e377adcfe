"""Test oracles: independent Python implementations the native exporter is cross-checked against.

They are NOT part of the shipped exporter: the image's `gpumon serve` imports none
of them, and grpcio / protobuf are only needed here.
  attribution/  grpcio CRI + PodResources clients, the Python control plane, the fake kubelet
                (gRPC server the native grpc_lite clients and the doctor are tested against)
  ops/pmc.py    Python derivation of the PMC series (parity oracle for csrc/core/ondevice.cpp)
  ops/probe.py  Python runner of the K1 probe plugin
"""
