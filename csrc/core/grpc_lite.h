// Minimal unary gRPC client over HTTP/2 cleartext on a unix socket, plus a protobuf wire reader.
//
// Enough for the kubelet PodResources API (/var/lib/kubelet/pod-resources/kubelet.sock) so the
// standalone native exporter (bin/gpumon-exporter) can attribute idle GPU allocations without the
// Python control plane or a gRPC library. The reference got the same information by `docker exec`
// into every opted-in container and running `nvidia-smi -L` there (gpu.py:220-253).
//
// HTTP/2 subset: prior-knowledge preface, SETTINGS (+ACK), PING ACK, one request stream with
// HPACK literal (never-indexed, non-Huffman) request headers, a 16 MiB receive window so large
// responses need no WINDOW_UPDATE round-trips, DATA reassembly, RST_STREAM/GOAWAY as errors.
// Response headers and trailers (HEADERS + CONTINUATION) are HPACK-decoded (hpack.h): the call's
// :status, grpc-status and grpc-message decide success, so Unimplemented / PermissionDenied /
// version skew from the kubelet or the runtime are reported as such.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <string_view>
#include <vector>

namespace gpumon {

// Outcome of a call as the server reported it.
struct GrpcStatus {
  int code = -1;          // grpc-status (0 OK ... 16 UNAUTHENTICATED); -1 = none received (transport failure)
  std::string message;    // grpc-message, percent-decoded
  int http_status = 0;    // :status of the response headers
};
const char* grpc_code_name(int code);  // "UNIMPLEMENTED", ... ("UNKNOWN_CODE" out of range)
// "%XX" sequences of a grpc-message value decoded (gRPC over HTTP/2 spec).
std::string grpc_percent_decode(std::string_view s);

// Unary call: `path` like "/v1.PodResourcesLister/List", `request` = serialized protobuf. False
// with `err` = "grpc-status 12 UNIMPLEMENTED: <message>" (or the transport failure) unless the
// server answered OK with a message; `status` (optional) receives the server's verdict either way.
bool grpc_unary_unix(const std::string& socket_path, const std::string& path, const std::string& request,
                     std::string* response, std::string* err, int timeout_ms = 3000, GrpcStatus* status = nullptr);

// Protobuf wire-format reader (varint / length-delimited; fixed32/64 skipped).
class PbReader {
 public:
  explicit PbReader(std::string_view b) : b_(b) {}
  // Next field; false at end or on malformed input (then ok() is false).
  bool next(uint32_t* field, uint32_t* wire);
  bool varint(uint64_t* v);
  bool bytes(std::string_view* v);
  bool skip(uint32_t wire);
  bool ok() const { return ok_; }

 private:
  std::string_view b_;
  size_t p_ = 0;
  bool ok_ = true;
};

// kubelet PodResources v1: every (pod, container, resource, device id) of `resource_prefix`
// resources (e.g. "amd.com/gpu").
struct PodDeviceRow {
  std::string pod_namespace, pod_name, container_name, resource_name, device_id;
};
// Device-plugin rows whose resource starts with `resource_prefix`, plus DRA claim devices
// (ContainerResources.dynamic_resources) of the drivers in `dra_drivers` (resource_name = driver,
// device_id = its device name, else the first CDI device name).
bool podresources_list(const std::string& socket_path, const std::string& resource_prefix,
                       std::vector<PodDeviceRow>* out, std::string* err, int timeout_ms = 3000,
                       const std::vector<std::string>& dra_drivers = {}, GrpcStatus* status = nullptr);
bool parse_list_pod_resources(std::string_view msg, const std::string& resource_prefix,
                              std::vector<PodDeviceRow>* out, const std::vector<std::string>& dra_drivers = {});

// CRI runtime.v1 RuntimeService ListContainers + ListPodSandbox (containerd / cri-o): container id
// -> pod identity and labels (the reference read the same io.kubernetes.* labels with
// `docker inspect`, gpu.py:86-88,184-195).
struct CriContainer {
  std::string id, sandbox_id, name;
  std::map<std::string, std::string> labels, annotations;
};
struct CriSandbox {
  std::string id, name, uid, pod_namespace;
  std::map<std::string, std::string> labels, annotations;
};
bool parse_cri_containers(std::string_view msg, std::vector<CriContainer>* out);
bool parse_cri_sandboxes(std::string_view msg, std::vector<CriSandbox>* out);
bool cri_list(const std::string& socket_path, std::vector<CriContainer>* containers, std::vector<CriSandbox>* sandboxes,
              std::string* err, int timeout_ms = 3000, GrpcStatus* status = nullptr);

}  // namespace gpumon
