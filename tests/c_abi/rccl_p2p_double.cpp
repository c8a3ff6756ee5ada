// Test double of the RCCL point-to-point subset sa_rccl.cpp uses, for a CPU
// test of the `direct` exchange's and the gather's slot arithmetic with W
// ranks (tests/test_rccl_p2p_double.py).  RCCL refuses two ranks on one GPU
// and no multi-GPU box is ours, so sa_comm_alltoall_u64 / sa_comm_gather_f64
// are linked here against this double instead of librccl: every rank is a
// thread, buffers are host memory, ncclSend/ncclRecv inside a group are
// matched per (source, destination) in issue order when the group ends, and
// a receive whose size differs from the matching send, a send never received
// or a receive never sent fails the run (RCCL would hang or corrupt there).
//
// Not a product file: only the test links it (no librccl, no HIP runtime).
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/sfl_sa.h"

void sa_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  fprintf(stderr, "sa_set_error: ");
  vfprintf(stderr, fmt, ap);
  fprintf(stderr, "\n");
  va_end(ap);
}

namespace {

struct Msg {
  const void* p;
  size_t bytes;
  bool* done;
};

struct World {
  int n = 0;
  std::mutex m;
  std::condition_variable cv;
  std::map<std::pair<int, int>, std::deque<Msg>> box;  // (src, dst) -> posted sends
};

struct Comm {
  World* w;
  int rank;
};

struct Op {
  bool send;
  int peer;
  void* p;
  size_t bytes;
};

thread_local int g_depth = 0;
thread_local Comm* g_comm = nullptr;
thread_local std::vector<Op> g_ops;

size_t type_bytes(ncclDataType_t t) {
  switch (t) {
    case ncclUint64:
    case ncclInt64:
    case ncclFloat64:
      return 8;
    default:
      return 4;
  }
}

[[noreturn]] void die(const char* what, int rank) {
  fprintf(stderr, "rccl double: rank %d: %s\n", rank, what);
  fflush(stderr);
  std::_Exit(3);
}

void flush_group() {
  Comm* c = g_comm;
  if (!c) {
    g_ops.clear();
    return;
  }
  World* w = c->w;
  std::vector<bool*> mine;
  {
    std::lock_guard<std::mutex> lk(w->m);
    for (const Op& o : g_ops)
      if (o.send) {
        bool* d = new bool(false);
        mine.push_back(d);
        w->box[{c->rank, o.peer}].push_back({o.p, o.bytes, d});
      }
  }
  w->cv.notify_all();
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(20);
  for (const Op& o : g_ops) {
    if (o.send) continue;
    std::unique_lock<std::mutex> lk(w->m);
    auto& q = w->box[{o.peer, c->rank}];
    if (!w->cv.wait_until(lk, deadline, [&] { return !q.empty(); }))
      die("a receive was never matched by a send (RCCL would hang)", c->rank);
    Msg msg = q.front();
    q.pop_front();
    if (msg.bytes != o.bytes) die("receive size differs from the matching send", c->rank);
    memcpy(o.p, msg.p, o.bytes);
    *msg.done = true;
    lk.unlock();
    w->cv.notify_all();
  }
  for (bool* d : mine) {
    std::unique_lock<std::mutex> lk(w->m);
    if (!w->cv.wait_until(lk, deadline, [&] { return *d; }))
      die("a send was never received (RCCL would hang)", c->rank);
  }
  for (bool* d : mine) delete d;
  g_ops.clear();
  g_comm = nullptr;
}

ncclResult_t post(bool send, void* p, size_t count, ncclDataType_t t, int peer, ncclComm_t comm) {
  Comm* c = reinterpret_cast<Comm*>(comm);
  if (peer < 0 || peer >= c->w->n || peer == c->rank) die("send/recv to an invalid peer", c->rank);
  if (g_comm && g_comm != c) die("one group across two communicators", c->rank);
  g_comm = c;
  g_ops.push_back({send, peer, p, count * type_bytes(t)});
  if (g_depth == 0) flush_group();
  return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGroupStart() {
  ++g_depth;
  return ncclSuccess;
}
ncclResult_t ncclGroupEnd() {
  if (--g_depth == 0) flush_group();
  return ncclSuccess;
}
ncclResult_t ncclSend(const void* p, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t) {
  return post(true, const_cast<void*>(p), count, t, peer, comm);
}
ncclResult_t ncclRecv(void* p, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t) {
  return post(false, p, count, t, peer, comm);
}
ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  *rank = reinterpret_cast<Comm*>(comm)->rank;
  return ncclSuccess;
}
ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  *count = reinterpret_cast<Comm*>(comm)->w->n;
  return ncclSuccess;
}
ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* device) {
  *device = reinterpret_cast<Comm*>(comm)->rank;  // one device per rank thread
  return ncclSuccess;
}
const char* ncclGetErrorString(ncclResult_t) { return "rccl double"; }
// collectives and set-up sa_rccl.cpp references but this test does not call
ncclResult_t ncclGetUniqueId(ncclUniqueId*) { return ncclInternalError; }
ncclResult_t ncclCommInitRank(ncclComm_t*, int, ncclUniqueId, int) { return ncclInternalError; }
ncclResult_t ncclCommDestroy(ncclComm_t) { return ncclSuccess; }
ncclResult_t ncclReduce(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t, hipStream_t) {
  return ncclInternalError;
}
ncclResult_t ncclAllReduce(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) {
  return ncclInternalError;
}
ncclResult_t ncclReduceScatter(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) {
  return ncclInternalError;
}
// the root's own-shard copy of sa_comm_gather_f64 (host memory here)
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes, hipMemcpyKind, hipStream_t) {
  memcpy(dst, src, bytes);
  return hipSuccess;
}
hipError_t hipSetDevice(int) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "hip double"; }

}  // extern "C"

// ---------------------------------------------------------------- the test
//
// W ranks, count elements per slot.  Rank r's send buffer holds value
// tag(r, p, i) in slot p; after sa_comm_alltoall_u64 rank r's recv slot p
// (p != r) must hold tag(p, r, i) -- rank p's shard r -- and slot r must be
// untouched.  Then sa_comm_gather_f64 to every root in turn.
static uint64_t tag(int src, int slot, uint64_t i) {
  return (uint64_t(src) << 56) ^ (uint64_t(slot) << 48) ^ (i * 0x9E3779B97F4A7C15ull);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s WORLD COUNT\n", argv[0]);
    return 2;
  }
  const int W = atoi(argv[1]);
  const uint64_t count = strtoull(argv[2], nullptr, 10);
  World world;
  world.n = W;
  std::vector<Comm> comms(W);
  for (int r = 0; r < W; ++r) comms[r] = {&world, r};
  std::vector<int> bad(W, 0);
  std::vector<std::thread> ts;
  for (int r = 0; r < W; ++r)
    ts.emplace_back([&, r] {
      std::vector<uint64_t> send(W * count), recv(W * count, ~0ull);
      for (int p = 0; p < W; ++p)
        for (uint64_t i = 0; i < count; ++i) send[p * count + i] = tag(r, p, i);
      if (sa_comm_alltoall_u64(&comms[r], send.data(), recv.data(), count, nullptr) != SA_OK) bad[r] |= 1;
      int nr = -1, rk = -1, dv = -1;  // sa_comm_info: what the communicator says of itself
      if (sa_comm_info(&comms[r], &nr, &rk, &dv) != SA_OK || nr != W || rk != r || dv != r) bad[r] |= 8;
      if (sa_comm_info(&comms[r], nullptr, nullptr, nullptr) != SA_OK) bad[r] |= 8;
      for (int p = 0; p < W; ++p)
        for (uint64_t i = 0; i < count; ++i) {
          uint64_t want = p == r ? ~0ull : tag(p, r, i);
          if (recv[p * count + i] != want) bad[r] |= 2;
        }
      for (int root = 0; root < W; ++root) {
        std::vector<double> mine(count), all(r == root ? W * count : 0, -1.0);
        for (uint64_t i = 0; i < count; ++i) mine[i] = double(r) * 1e6 + double(i) + 0.25 * root;
        if (sa_comm_gather_f64(&comms[r], mine.data(), r == root ? all.data() : nullptr, count, root, nullptr) != SA_OK)
          bad[r] |= 4;
        if (r == root)
          for (int p = 0; p < W; ++p)
            for (uint64_t i = 0; i < count; ++i)
              if (all[p * count + i] != double(p) * 1e6 + double(i) + 0.25 * root) bad[r] |= 8;
      }
    });
  for (auto& t : ts) t.join();
  int rc = 0;
  for (int r = 0; r < W; ++r)
    if (bad[r]) {
      fprintf(stderr, "rank %d: failures 0x%x (1 alltoall call, 2 alltoall slots, 4 gather call, 8 gather slots)\n",
              r, bad[r]);
      rc = 1;
    }
  if (!rc) printf("ok world=%d count=%llu\n", W, (unsigned long long)count);
  return rc;
}
