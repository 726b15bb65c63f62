// TEST INFRASTRUCTURE ONLY: an in-process loopback stand-in for RCCL's point-to-point API (SURVEY
// §4 item 5: "an in-process loopback communicator behind the same interface as RCCL"), so that
// the distinct-device exchange of kh_trie_root_sharded (csrc/sharded.h: ncclCommInitAll, grouped
// ncclSend / ncclRecv of the keys on each shard's build stream, then the lengths and values on
// its exchange stream) runs on the one-GPU box, where real RCCL refuses a device list that
// repeats a device.
//
// Exports the six symbols sharded.h resolves (ncclCommInitAll, ncclGroupStart, ncclGroupEnd,
// ncclSend, ncclRecv, ncclGetErrorString) under the soname librccl.so, so a process that loads it
// with RTLD_GLOBAL before its first sharded call has sharded.h's RTLD_NOLOAD lookup find it.
//   - communicators: one per listed device, repeats allowed (rank g = position g);
//   - a group's operations are matched at ncclGroupEnd: the k-th send from rank g to rank p with
//     the k-th receive on rank p from rank g; a send or receive without its partner, a size or
//     element-type mismatch, or a peer outside the communicator fails the group
//     (ncclInvalidUsage) and nothing is copied;
//   - each matched pair is one copy on the RECEIVER's stream after the sender's stream has
//     reached the send (an event), and the sender's stream waits for the copy's completion (an
//     event), so both streams see the operation as RCCL's do: later work on either waits for it;
//   - loopback_stats() reports the matched operations and bytes, so a test can tell that the
//     exchange really went through here.
// Build: hipcc -shared -fPIC -O2 -Wl,-soname,librccl.so -o librccl.so loopback_rccl.cpp
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

struct ncclComm {
  int rank, nranks;
  const std::vector<int>* devs;  // the communicator set's devices by rank (repeats allowed)
};

namespace {
struct Op {
  bool send;
  void* buf;
  size_t bytes;
  ncclDataType_t type;
  int self, peer;
  hipStream_t st;
  const std::vector<int>* devs;
};
std::mutex g_mu;
int g_depth = 0;
std::vector<Op> g_ops;
uint64_t g_ops_matched = 0, g_bytes = 0, g_groups = 0;

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8:
    case ncclUint8:
      return 1;
    case ncclFloat16:
    case ncclBfloat16:
      return 2;
    case ncclInt32:
    case ncclUint32:
    case ncclFloat32:
      return 4;
    case ncclInt64:
    case ncclUint64:
    case ncclFloat64:
      return 8;
    default:
      return 0;
  }
}

ncclResult_t run_group(std::vector<Op>& ops) {
  // k-th send g->p with the k-th recv at p from g
  std::map<std::pair<int, int>, std::vector<const Op*>> sends, recvs;
  for (const Op& o : ops) (o.send ? sends : recvs)[o.send ? std::make_pair(o.self, o.peer) : std::make_pair(o.peer, o.self)].push_back(&o);
  if (sends.size() != recvs.size()) return ncclInvalidUsage;
  for (auto& kv : sends) {
    auto it = recvs.find(kv.first);
    if (it == recvs.end() || it->second.size() != kv.second.size()) return ncclInvalidUsage;
    for (size_t k = 0; k < kv.second.size(); ++k)
      if (kv.second[k]->bytes != it->second[k]->bytes || kv.second[k]->type != it->second[k]->type) return ncclInvalidUsage;
  }
  for (auto& kv : sends) {
    const auto& rv = recvs[kv.first];
    for (size_t k = 0; k < kv.second.size(); ++k) {
      const Op& s = *kv.second[k];
      const Op& r = *rv[k];
      if (s.devs != r.devs) return ncclInvalidUsage;  // (two communicator sets)
      const std::vector<int>& devs = *s.devs;
      if (!s.bytes) continue;
      hipEvent_t sent, done;
      if (hipSetDevice(devs[s.self]) != hipSuccess) return ncclInternalError;
      if (hipEventCreateWithFlags(&sent, hipEventDisableTiming) != hipSuccess) return ncclInternalError;
      if (hipEventRecord(sent, s.st) != hipSuccess) return ncclInternalError;
      if (hipSetDevice(devs[r.self]) != hipSuccess) return ncclInternalError;
      if (hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) return ncclInternalError;
      if (hipStreamWaitEvent(r.st, sent, 0) != hipSuccess) return ncclInternalError;
      if (hipMemcpyPeerAsync(r.buf, devs[r.self], s.buf, devs[s.self], s.bytes, r.st) != hipSuccess)
        return ncclUnhandledCudaError;
      if (hipEventRecord(done, r.st) != hipSuccess) return ncclInternalError;
      if (hipSetDevice(devs[s.self]) != hipSuccess) return ncclInternalError;
      if (hipStreamWaitEvent(s.st, done, 0) != hipSuccess) return ncclInternalError;
      (void)hipEventDestroy(sent);  // (released once the streams are past them)
      (void)hipEventDestroy(done);
      g_ops_matched += 2;
      g_bytes += s.bytes;
    }
  }
  return ncclSuccess;
}
}  // namespace

extern "C" {

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
  if (!comms || ndev < 1 || !devlist) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(g_mu);
  const std::vector<int>* set = new std::vector<int>(devlist, devlist + ndev);  // (kept for the process)
  for (int g = 0; g < ndev; ++g) comms[g] = new ncclComm{g, ndev, set};
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  std::lock_guard<std::mutex> lk(g_mu);
  ++g_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_depth <= 0) return ncclInvalidUsage;
  if (--g_depth) return ncclSuccess;
  std::vector<Op> ops;
  ops.swap(g_ops);
  int cur = 0;
  (void)hipGetDevice(&cur);
  const ncclResult_t r = run_group(ops);
  (void)hipSetDevice(cur);
  ++g_groups;
  return r;
}

static ncclResult_t post(bool send, const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                         hipStream_t st) {
  if (!comm || peer < 0 || peer >= comm->nranks || type_size(t) == 0) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_depth <= 0) return ncclInvalidUsage;  // (sharded.h always groups its operations)
  g_ops.push_back(Op{send, (void*)buf, count * type_size(t), t, comm->rank, peer, st, comm->devs});
  return ncclSuccess;
}
ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t st) {
  return post(true, buf, count, t, peer, comm, st);
}
ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t st) {
  return post(false, buf, count, t, peer, comm, st);
}

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess:
      return "no error (loopback)";
    case ncclInvalidArgument:
      return "invalid argument (loopback)";
    case ncclInvalidUsage:
      return "invalid usage: unmatched send/recv or size mismatch (loopback)";
    default:
      return "internal error (loopback)";
  }
}

// test hook: matched operations (sends + receives), bytes copied, groups completed
void loopback_stats(uint64_t* ops, uint64_t* bytes, uint64_t* groups) {
  std::lock_guard<std::mutex> lk(g_mu);
  *ops = g_ops_matched;
  *bytes = g_bytes;
  *groups = g_groups;
}
}
