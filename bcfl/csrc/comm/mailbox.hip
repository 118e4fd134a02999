// One-sided peer mailboxes for truly asynchronous P2P gossip over xGMI.
//
// The reference's "P2P" is an in-process host average (src/Serverlesscase/serverless_NonIID_IMDB.py:
// 284-297); its paper claims asynchronous exchange (README.md:10, async = max over destinations in
// Medical_Transcriptions_All_graphs.ipynb:979-980). RCCL send/recv needs a matched receive on the
// peer, so a slow or dead peer stalls the sender. Here every receiver owns, per remote client it
// listens to, an INBOX: one dedicated hipMalloc region
//
//     [ header slot 0 | header slot 1 | pad to 4 KiB | payload slot 0 | payload slot 1 ]
//
// exported once with hipIpcGetMemHandle and mapped by the sender with hipIpcOpenMemHandle. The
// sender of version v writes slot v % 2 with three stream-ordered operations on its own side
// stream: header.begin = v (this kernel), payload copy (hipMemcpyAsync over xGMI, issued from
// Python), then header.{round, steps, root, ...} and header.end = v (this kernel, with a
// system-scope fence between the body words and the end word). A reader takes the newest slot
// whose begin == end, copies it into local memory and re-reads the header: if begin moved the
// sender lapped the slot mid-copy and the snapshot is discarded (seqlock). No receive is ever
// posted, nothing waits for a peer.
//
// Header slot layout (int64 x 16 = 128 B, one line per slot):
//   [0] begin version  [1] round  [2] steps  [3] payload bytes  [4..7] SHA-256 Merkle root
//   [8] end version    [9..15] reserved
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "mailbox.h"

namespace bcfl_comm {

using torch::Tensor;

namespace {

void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "mailbox ", what, ": ", hipGetErrorString(e));
}

constexpr int kHdrWords = 16;

// one wave; lane i < n writes word off + i. The end word is written by lane 0 after a
// system-scope fence so a reader that sees end == v also sees the body words.
__global__ void hdr_store_kernel(int64_t* __restrict__ hdr, int off, int n, int64_t w0,
                                 int64_t w1, int64_t w2, int64_t w3, int64_t w4, int64_t w5,
                                 int64_t w6, int end_word, int64_t end_value) {
  const int i = threadIdx.x;
  int64_t v = 0;
  switch (i) {
    case 0: v = w0; break;
    case 1: v = w1; break;
    case 2: v = w2; break;
    case 3: v = w3; break;
    case 4: v = w4; break;
    case 5: v = w5; break;
    case 6: v = w6; break;
    default: break;
  }
  if (i < n) hdr[off + i] = v;
  __threadfence_system();
  __syncthreads();
  if (end_word >= 0 && i == 0) {
    __hip_atomic_store(hdr + end_word, end_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace

// flags: hipDeviceMallocDefault (0) or hipDeviceMallocUncached (3). Mailboxes are written by a
// PEER over xGMI and read by this GPU: coarse-grained memory is only coherent at kernel
// boundaries of the writer/reader pair on ONE device, so headers (and by default payloads) live
// in uncached memory where every access goes to HBM and a peer's completed write is always seen.
Tensor mbox_alloc(int64_t nbytes, int64_t device, int64_t flags) {
  TORCH_CHECK(nbytes > 0, "mailbox size must be positive");
  TORCH_CHECK(flags == hipDeviceMallocDefault || flags == hipDeviceMallocUncached ||
                  flags == hipDeviceMallocFinegrained,
              "unsupported mailbox allocation flags ", flags);
  int prev = 0;
  hip_check(hipGetDevice(&prev), "hipGetDevice");
  hip_check(hipSetDevice((int)device), "hipSetDevice");
  void* p = nullptr;
  if (flags == hipDeviceMallocDefault) {
    hip_check(hipMalloc(&p, (size_t)nbytes), "hipMalloc");
  } else {
    hip_check(hipExtMallocWithFlags(&p, (size_t)nbytes, (unsigned)flags), "hipExtMallocWithFlags");
  }
  hip_check(hipMemset(p, 0, (size_t)nbytes), "hipMemset");
  hip_check(hipSetDevice(prev), "hipSetDevice");
  auto opts = torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, (int)device);
  return torch::from_blob(p, {nbytes}, [](void* q) { (void)hipFree(q); }, opts);
}

pybind11::bytes ipc_handle(Tensor t) {
  TORCH_CHECK(t.is_cuda(), "ipc_handle needs a GPU tensor");
  void* base = nullptr;
  size_t size = 0;
  hip_check(hipMemGetAddressRange(&base, &size, t.data_ptr()), "hipMemGetAddressRange");
  TORCH_CHECK(base == t.data_ptr(), "ipc_handle: tensor must start its own allocation (use mbox_alloc)");
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, t.data_ptr()), "hipIpcGetMemHandle");
  return pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
}

// Can `device` read and write memory that lives on `peer` (xGMI / PCIe peer-to-peer)? Every
// mailbox post is a copy issued on the sender's device into the receiver's HBM.
bool can_access_peer(int64_t device, int64_t peer) {
  if (device == peer) return true;
  int n = 0;
  hip_check(hipGetDeviceCount(&n), "hipGetDeviceCount");
  TORCH_CHECK(device >= 0 && device < n && peer >= 0 && peer < n, "can_access_peer: device ",
              device, " / peer ", peer, " outside the ", n, " visible devices");
  int ok = 0;
  hip_check(hipDeviceCanAccessPeer(&ok, (int)device, (int)peer), "hipDeviceCanAccessPeer");
  return ok != 0;
}

// peer_device >= 0: the device that owns the exported allocation; mapping it for use on
// `device` needs peer access between the two (checked first: without it the lazily enabled peer
// mapping would fail later, inside a copy)
Tensor ipc_open(const std::string& handle, int64_t nbytes, int64_t device, int64_t peer_device) {
  TORCH_CHECK(handle.size() == sizeof(hipIpcMemHandle_t), "bad IPC handle size");
  if (peer_device >= 0 && peer_device != device) {
    TORCH_CHECK(can_access_peer(device, peer_device), "mailbox: device ", device,
                " has no peer access to device ", peer_device,
                " (hipDeviceCanAccessPeer = 0: no xGMI / PCIe P2P path)");
  }
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  int prev = 0;
  hip_check(hipGetDevice(&prev), "hipGetDevice");
  hip_check(hipSetDevice((int)device), "hipSetDevice");
  void* p = nullptr;
  hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  hip_check(hipSetDevice(prev), "hipSetDevice");
  auto opts = torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, (int)device);
  return torch::from_blob(p, {nbytes}, [](void* q) { (void)hipIpcCloseMemHandle(q); }, opts);
}

void hdr_store(Tensor hdr, int64_t slot, std::vector<int64_t> words, int64_t off, int64_t end_word,
               int64_t end_value) {
  TORCH_CHECK(hdr.is_cuda() && hdr.scalar_type() == torch::kInt64, "header must be GPU int64");
  TORCH_CHECK(hdr.numel() >= 2 * kHdrWords, "header view too small");
  TORCH_CHECK(words.size() <= 7 && off >= 0 && off + (int64_t)words.size() <= kHdrWords,
              "header words out of range");
  TORCH_CHECK(end_word < kHdrWords && slot >= 0 && slot < 2, "header slot / end word out of range");
  int64_t w[7] = {0, 0, 0, 0, 0, 0, 0};
  for (size_t i = 0; i < words.size(); ++i) w[i] = words[i];
  int64_t* base = hdr.data_ptr<int64_t>() + slot * kHdrWords;
  hipLaunchKernelGGL(hdr_store_kernel, dim3(1), dim3(64), 0,
                     c10::hip::getCurrentHIPStream().stream(), base, (int)off, (int)words.size(),
                     w[0], w[1], w[2], w[3], w[4], w[5], w[6], (int)end_word, end_value);
  hip_check(hipGetLastError(), "hdr_store launch");
}

void register_mailbox(pybind11::module& m) {
  m.def("mbox_alloc", &mbox_alloc, "dedicated device allocation (IPC-exportable), zeroed",
        pybind11::arg("nbytes"), pybind11::arg("device"), pybind11::arg("flags") = 3);
  m.def("ipc_handle", &ipc_handle, "hipIpcGetMemHandle of an mbox_alloc tensor");
  m.def("ipc_open", &ipc_open, "map a peer's mailbox (hipIpcOpenMemHandle) as a uint8 tensor",
        pybind11::arg("handle"), pybind11::arg("nbytes"), pybind11::arg("device"),
        pybind11::arg("peer_device") = -1);
  m.def("can_access_peer", &can_access_peer, "hipDeviceCanAccessPeer(device, peer)");
  m.def("hdr_store", &hdr_store, "stream-ordered header word store (+ fenced end word)");
}

}  // namespace bcfl_comm
