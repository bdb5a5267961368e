// comm.cpp -- frontier exchange between ranks: the multi-GPU replacement of StorageClient's
// per-host RPC scatter/gather (src/storage/client/StorageClient.inl:74-159).
//
// Two transports behind one interface:
//   * RCCL over xGMI (production): one process per GPU; collectives are issued on the
//     context's stream so they order with the expansion kernels.  Variable-size exchanges use
//     grouped ncclSend/ncclRecv: on MI355X every peer pair has its own xGMI link, so the 7
//     transfers of an 8-GPU exchange run concurrently (all-to-all, not ring).
//   * LocalGroup (tests): several contexts of one process on one device form a group; the same
//     collective calls become device-to-device copies between the ranks' buffers, so the
//     sharded algorithm runs unchanged with N ranks on a single GPU.
#include <rccl/rccl.h>

#include <condition_variable>
#include <map>
#include <mutex>
#include <vector>

#include "engine.h"

namespace nbg {

#define NBG_NCCL(x)                                                                                \
  do {                                                                                             \
    ncclResult_t r_ = (x);                                                                         \
    if (r_ != ncclSuccess) throw Error(NBG_E_COMM, std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

struct CommImpl {
  virtual ~CommImpl() = default;
  // every rank contributes `send` (send_bytes) into recv + recv_off[r] of every rank
  virtual void allgatherv(Ctx& c, const void* send, size_t send_bytes, void* recv, const size_t* recv_bytes,
                          const size_t* recv_off) = 0;
  virtual void alltoallv(Ctx& c, const void* send, const size_t* send_bytes, const size_t* send_off, void* recv,
                         const size_t* recv_bytes, const size_t* recv_off) = 0;
  virtual void allreduce_sum_i64(Ctx& c, int64_t* d, size_t n) = 0;
  // allgatherv plus a small fixed-size allgather in the same exchange (one grouped launch):
  // every rank's send2 (bytes2) lands at recv2 + r * bytes2 of every rank
  virtual void allgatherv2(Ctx& c, const void* send, size_t send_bytes, void* recv, const size_t* recv_bytes,
                           const size_t* recv_off, const void* send2, size_t bytes2, void* recv2) = 0;
  virtual int32_t ranks() const = 0;     // the communicator's own rank count
  virtual int32_t transport() const = 0;  // 1 = RCCL, 2 = in-process LocalComm
};

// ------------------------------------------------------------------------------------------
struct RcclComm : CommImpl {
  ncclComm_t comm = nullptr;
  // self_p2p: the rank's own slice also goes through ncclSend / ncclRecv to itself (a one-rank
  // communicator, option comm_single, runs every RCCL entry point on a one-GPU box); otherwise it
  // is a device-to-device copy beside the grouped transfers
  bool self_p2p = false;
  int32_t ranks() const override {
    int n = 0;
    return ncclCommCount(comm, &n) == ncclSuccess ? int32_t(n) : -1;
  }
  int32_t transport() const override { return 1; }
  ~RcclComm() override {
    if (comm) ncclCommDestroy(comm);
  }
  bool skip(const Ctx& c, int p) const { return p == c.rank && !self_p2p; }
  void self_copy(Ctx& c, void* dst, const void* src, size_t bytes) {
    if (!self_p2p && bytes && dst != src) NBG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c.stream));
  }
  // point-to-point transfers in pieces of at most msg bytes (option comm_chunk_mb, default 1024):
  // both sides split a transfer identically, and RCCL pairs the pieces of one peer pair in issue
  // order (see DESIGN.md section 4 for the measured reason)
  size_t msg = size_t(1) << 30;
  void p2p_send(const void* buf, size_t bytes, int peer, hipStream_t s) {
    for (size_t o = 0; o < bytes; o += msg)
      NBG_NCCL(ncclSend(static_cast<const uint8_t*>(buf) + o, std::min(msg, bytes - o), ncclUint8, peer, comm, s));
  }
  void p2p_recv(void* buf, size_t bytes, int peer, hipStream_t s) {
    for (size_t o = 0; o < bytes; o += msg)
      NBG_NCCL(ncclRecv(static_cast<uint8_t*>(buf) + o, std::min(msg, bytes - o), ncclUint8, peer, comm, s));
  }
  void allgatherv(Ctx& c, const void* send, size_t send_bytes, void* recv, const size_t* recv_bytes,
                  const size_t* recv_off) override {
    NBG_NCCL(ncclGroupStart());
    for (int p = 0; p < c.world; p++) {
      if (skip(c, p)) continue;
      if (p == c.rank && static_cast<uint8_t*>(recv) + recv_off[p] == send) {
        // in place: the own slice is already where it belongs
      } else {
        p2p_send(send, send_bytes, p, c.stream);
        p2p_recv(static_cast<uint8_t*>(recv) + recv_off[p], recv_bytes[p], p, c.stream);
      }
    }
    NBG_NCCL(ncclGroupEnd());
    self_copy(c, static_cast<uint8_t*>(recv) + recv_off[c.rank], send, send_bytes);
  }
  void alltoallv(Ctx& c, const void* send, const size_t* send_bytes, const size_t* send_off, void* recv,
                 const size_t* recv_bytes, const size_t* recv_off) override {
    NBG_NCCL(ncclGroupStart());
    for (int p = 0; p < c.world; p++) {
      if (skip(c, p)) continue;
      p2p_send(static_cast<const uint8_t*>(send) + send_off[p], send_bytes[p], p, c.stream);
      p2p_recv(static_cast<uint8_t*>(recv) + recv_off[p], recv_bytes[p], p, c.stream);
    }
    NBG_NCCL(ncclGroupEnd());
    self_copy(c, static_cast<uint8_t*>(recv) + recv_off[c.rank], static_cast<const uint8_t*>(send) + send_off[c.rank],
              send_bytes[c.rank]);
  }
  void allreduce_sum_i64(Ctx& c, int64_t* d, size_t n) override {
    NBG_NCCL(ncclAllReduce(d, d, n, ncclInt64, ncclSum, comm, c.stream));
  }
  void allgatherv2(Ctx& c, const void* send, size_t send_bytes, void* recv, const size_t* recv_bytes,
                   const size_t* recv_off, const void* send2, size_t bytes2, void* recv2) override {
    NBG_NCCL(ncclGroupStart());
    for (int p = 0; p < c.world; p++) {
      if (skip(c, p)) continue;
      if (p == c.rank && static_cast<uint8_t*>(recv) + recv_off[p] == send) {
        // in place: the own slice is already where it belongs
      } else {
        p2p_send(send, send_bytes, p, c.stream);
        p2p_recv(static_cast<uint8_t*>(recv) + recv_off[p], recv_bytes[p], p, c.stream);
      }
      p2p_send(send2, bytes2, p, c.stream);
      p2p_recv(static_cast<uint8_t*>(recv2) + size_t(p) * bytes2, bytes2, p, c.stream);
    }
    NBG_NCCL(ncclGroupEnd());
    self_copy(c, static_cast<uint8_t*>(recv) + recv_off[c.rank], send, send_bytes);
    self_copy(c, static_cast<uint8_t*>(recv2) + size_t(c.rank) * bytes2, send2, bytes2);
  }
};

// ------------------------------------------------------------------------------------------
// In-process rank group, stream-ordered like RCCL: no collective waits for the GPU on the host.
// Each collective is three steps:
//   1. every rank records `ready` on its stream (its send buffer is complete) and publishes the
//      buffer pointers; host barrier A (only the enqueue order is synchronised, not the GPU);
//   2. every rank makes its stream wait for every peer's `ready`, enqueues its receive copies
//      from the peers' buffers and records `done`; host barrier B;
//   3. every rank makes its stream wait for every peer's `done` (nobody overwrites a send buffer
//      a peer still reads).
// A rank re-records `ready` / `done` only after the next collective's barrier A, which every
// rank reaches after step 3 of this one, so one event pair per rank suffices.
struct LocalGroup {
  int world = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<const void*> ptr, ptr2;
  std::vector<const size_t*> sizes, offs, rsizes;
  std::vector<size_t> scalar;
  std::vector<uint64_t> op;  // per rank: the collective it entered (kind | fixed size << 8)
  std::vector<hipEvent_t> ready, done;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};
static std::mutex g_groups_mu;
static std::map<int64_t, std::shared_ptr<LocalGroup>> g_groups;

__global__ void k_sum_slices(const int64_t* in, int world, size_t n, int64_t* out) {
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) {
    int64_t s = 0;
    for (int p = 0; p < world; p++) s += in[size_t(p) * n + i];
    out[i] = s;
  }
}

// The in-process transport also holds every exchange to RCCL's pairing rule: a grouped
// ncclSend / ncclRecv pair must agree on the byte count, and a side that skips a zero-byte
// transfer must face a peer that skips it too (otherwise RCCL hangs or truncates); and every rank
// must be in the same collective (RCCL matches them by issue order).  Each rank publishes its
// collective, send sizes and receive sizes before barrier A; after it every rank checks every
// pair from the same published arrays, so all ranks reach the same verdict before any data moves.
// On a mismatch no rank copies anything (a peer's pointers may belong to another collective),
// every rank still passes barrier B so the group stays in step, and every rank throws.
struct LocalComm : CommImpl {
  int32_t transport() const override { return 2; }
  int32_t ranks() const override { return g ? int32_t(g->world) : -1; }
  std::shared_ptr<LocalGroup> g;
  hipEvent_t ready = nullptr, done = nullptr;
  DevBuf scratch;  // allreduce: every rank's slice, then the sums
  ~LocalComm() override {
    if (ready) (void)hipEventDestroy(ready);
    if (done) (void)hipEventDestroy(done);
  }
  // what rank p sends to rank q (kinds 1 and 3: the same to everyone; 2: its row of send sizes)
  size_t sent(int kind, int p, int q) const { return kind == 2 ? g->sizes[size_t(p)][q] : g->scalar[size_t(p)]; }
  // step 1 + barrier A, then the group's verdict (empty: every rank entered collective `op` and
  // every send pairs with its receive), the same string on every rank
  std::string publish(Ctx& c, uint64_t op, const size_t* recv_bytes) {
    g->op[size_t(c.rank)] = op;
    g->rsizes[size_t(c.rank)] = recv_bytes;
    NBG_HIP(hipEventRecord(ready, c.stream));
    g->barrier();
    for (int p = 0; p < c.world; p++)
      if (g->op[size_t(p)] != g->op[0])
        return "rank " + std::to_string(p) + " entered collective " + std::to_string(g->op[size_t(p)]) +
               " while rank 0 entered " + std::to_string(g->op[0]);
    const int kind = int(op & 0xFF);
    if (kind == 4) return std::string();  // allreduce: its size is part of op
    const char* what = kind == 1 ? "allgatherv" : kind == 2 ? "alltoallv" : "allgatherv2";
    for (int q = 0; q < c.world; q++)
      for (int p = 0; p < c.world; p++) {
        if (p == q) continue;
        const size_t sb = sent(kind, p, q), rb = g->rsizes[size_t(q)][p];
        if (sb != rb)
          return std::string(what) + ": rank " + std::to_string(p) + " sends " + std::to_string(sb) +
                 " bytes, rank " + std::to_string(q) + " receives " + std::to_string(rb);
      }
    return std::string();
  }
  // (after the receive copies, or none) step 2's `done` + barrier B + step 3, then the verdict
  void finish(Ctx& c, const std::string& mismatch) {
    NBG_HIP(hipEventRecord(done, c.stream));
    g->barrier();
    for (int p = 0; p < c.world; p++)
      if (p != c.rank) NBG_HIP(hipStreamWaitEvent(c.stream, g->done[size_t(p)], 0));
    if (!mismatch.empty()) throw Error(NBG_E_COMM, "exchange sizes would not pair under RCCL: " + mismatch);
  }
  void wait_ready(Ctx& c, int p) {
    if (p != c.rank) NBG_HIP(hipStreamWaitEvent(c.stream, g->ready[size_t(p)], 0));
  }
  void allgatherv(Ctx& c, const void* send, size_t send_bytes, void* recv, const size_t* recv_bytes,
                  const size_t* recv_off) override {
    g->ptr[size_t(c.rank)] = send;
    g->scalar[size_t(c.rank)] = send_bytes;
    const std::string bad = publish(c, 1, recv_bytes);
    for (int p = 0; p < c.world && bad.empty(); p++) {
      size_t b = std::min(g->scalar[size_t(p)], recv_bytes[p]);
      if (!b || g->ptr[size_t(p)] == static_cast<uint8_t*>(recv) + recv_off[p]) continue;
      wait_ready(c, p);
      NBG_HIP(hipMemcpyAsync(static_cast<uint8_t*>(recv) + recv_off[p], g->ptr[size_t(p)], b,
                             hipMemcpyDeviceToDevice, c.stream));
    }
    finish(c, bad);
  }
  void alltoallv(Ctx& c, const void* send, const size_t* send_bytes, const size_t* send_off, void* recv,
                 const size_t* recv_bytes, const size_t* recv_off) override {
    g->ptr[size_t(c.rank)] = send;
    g->sizes[size_t(c.rank)] = send_bytes;
    g->offs[size_t(c.rank)] = send_off;
    const std::string bad = publish(c, 2, recv_bytes);
    for (int p = 0; p < c.world && bad.empty(); p++) {
      size_t b = std::min(g->sizes[size_t(p)][c.rank], recv_bytes[p]);
      if (!b) continue;
      wait_ready(c, p);
      NBG_HIP(hipMemcpyAsync(static_cast<uint8_t*>(recv) + recv_off[p],
                             static_cast<const uint8_t*>(g->ptr[size_t(p)]) + g->offs[size_t(p)][c.rank], b,
                             hipMemcpyDeviceToDevice, c.stream));
    }
    finish(c, bad);
  }
  void allgatherv2(Ctx& c, const void* send, size_t send_bytes, void* recv, const size_t* recv_bytes,
                   const size_t* recv_off, const void* send2, size_t bytes2, void* recv2) override {
    g->ptr[size_t(c.rank)] = send;
    g->scalar[size_t(c.rank)] = send_bytes;
    g->ptr2[size_t(c.rank)] = send2;
    const std::string bad = publish(c, 3ull | uint64_t(bytes2) << 8, recv_bytes);
    for (int p = 0; p < c.world && bad.empty(); p++) {
      wait_ready(c, p);
      size_t b = std::min(g->scalar[size_t(p)], recv_bytes[p]);
      if (b && g->ptr[size_t(p)] != static_cast<uint8_t*>(recv) + recv_off[p])
        NBG_HIP(hipMemcpyAsync(static_cast<uint8_t*>(recv) + recv_off[p], g->ptr[size_t(p)], b,
                               hipMemcpyDeviceToDevice, c.stream));
      NBG_HIP(hipMemcpyAsync(static_cast<uint8_t*>(recv2) + size_t(p) * bytes2, g->ptr2[size_t(p)], bytes2,
                             hipMemcpyDeviceToDevice, c.stream));
    }
    finish(c, bad);
  }
  // in place, as ncclAllReduce: gather the slices, sum them, and write the sums back only after
  // every peer has read this rank's slice
  void allreduce_sum_i64(Ctx& c, int64_t* d, size_t n) override {
    if (n == 0) return;
    const size_t G = size_t(c.world);
    {
      PoolScope none(nullptr);  // owned by the communicator, outside the query pools
      scratch.ensure((G + 1) * n * 8);
    }
    int64_t* sl = scratch.as<int64_t>();
    g->ptr[size_t(c.rank)] = d;
    const std::string bad = publish(c, 4ull | uint64_t(n) << 8, nullptr);
    if (bad.empty()) {
      for (int p = 0; p < c.world; p++) {
        wait_ready(c, p);
        NBG_HIP(hipMemcpyAsync(sl + size_t(p) * n, g->ptr[size_t(p)], n * 8, hipMemcpyDeviceToDevice, c.stream));
      }
      k_sum_slices<<<1, 256, 0, c.stream>>>(sl, c.world, n, sl + G * n);
      NBG_HIP(hipGetLastError());
    }
    finish(c, bad);
    NBG_HIP(hipMemcpyAsync(d, sl + G * n, n * 8, hipMemcpyDeviceToDevice, c.stream));
  }
};

static CommImpl* impl(Ctx& c) {
  if (!c.comm) throw Error(NBG_E_STATE, "multi-rank context without a communicator (nbg_comm_init)");
  c.timing.comm_calls++;
  return static_cast<CommImpl*>(c.comm);
}

// ------------------------------------------------------------------------------------------
int32_t comm_unique_id(uint8_t out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return NBG_E_COMM;
  memcpy(out, &id, 128);
  return NBG_OK;
}

// world > 1: the rank's RCCL communicator.  world == 1: nothing, unless option comm_single = 1
// (set before the snapshot is built): then a one-rank RCCL communicator is formed and the
// context runs the sharded algorithm through it (every exchange, its own slice sent to itself)
void comm_init(Ctx& c, const uint8_t id_bytes[128]) {
  const bool single = c.world == 1 && c.opt("comm_single", 0) != 0;
  if (c.world == 1 && !single) return;
  if (c.comm) throw Error(NBG_E_STATE, "communicator already initialised");
  if (single && (c.finalized || c.n_global > 0))
    throw Error(NBG_E_STATE, "comm_single: initialise the communicator before the snapshot is built");
  ncclUniqueId id;
  memcpy(&id, id_bytes, 128);
  NBG_HIP(hipSetDevice(c.device));
  auto* r = new RcclComm();
  r->self_p2p = single;
  r->msg = size_t(std::max<int64_t>(1, c.opt("comm_chunk_mb", 1024))) << 20;
  pool_trim_all();  // RCCL's buffers come from the driver, which never trims the block caches
  ncclResult_t rc = ncclCommInitRank(&r->comm, c.world, id, c.rank);
  if (rc != ncclSuccess) {
    r->comm = nullptr;
    delete r;
    throw Error(NBG_E_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(rc));
  }
  c.comm = r;
  c.sharded = true;
}

void comm_init_local(Ctx& c, int64_t key) {
  if (c.world == 1) return;
  if (c.comm) throw Error(NBG_E_STATE, "communicator already initialised");
  std::shared_ptr<LocalGroup> g;
  {
    std::lock_guard<std::mutex> lk(g_groups_mu);
    auto& slot = g_groups[key];
    if (!slot) {
      slot = std::make_shared<LocalGroup>();
      slot->world = c.world;
      slot->ptr.resize(size_t(c.world));
      slot->ptr2.resize(size_t(c.world));
      slot->sizes.resize(size_t(c.world));
      slot->offs.resize(size_t(c.world));
      slot->rsizes.resize(size_t(c.world));
      slot->scalar.resize(size_t(c.world));
      slot->op.resize(size_t(c.world));
      slot->ready.resize(size_t(c.world));
      slot->done.resize(size_t(c.world));
    }
    g = slot;
  }
  if (g->world != c.world) throw Error(NBG_E_INVALID_ARG, "local group world size mismatch");
  auto* l = new LocalComm();
  l->g = g;
  if (hipEventCreateWithFlags(&l->ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&l->done, hipEventDisableTiming) != hipSuccess) {
    delete l;
    throw Error(NBG_E_DEVICE, "hipEventCreate (LocalComm)");
  }
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->ready[size_t(c.rank)] = l->ready;
    g->done[size_t(c.rank)] = l->done;
  }
  c.comm = l;
}

// (ranks, transport) of the context's communicator: what ncclCommCount reports for RCCL
void comm_info(const Ctx& c, int32_t* ranks, int32_t* transport) {
  auto* impl = static_cast<const CommImpl*>(c.comm);
  *ranks = impl ? impl->ranks() : 1;
  *transport = impl ? impl->transport() : 0;
}

void comm_destroy(Ctx& c) {
  delete static_cast<CommImpl*>(c.comm);
  c.comm = nullptr;
}

void comm_allgather_bytes(Ctx& c, const void* send, size_t bytes_each, void* recv) {
  if (!c.sharded) {
    NBG_HIP(hipMemcpyAsync(recv, send, bytes_each, hipMemcpyDeviceToDevice, c.stream));
    return;
  }
  std::vector<size_t> rb(size_t(c.world), bytes_each), ro(size_t(c.world));
  for (int p = 0; p < c.world; p++) ro[size_t(p)] = size_t(p) * bytes_each;
  impl(c)->allgatherv(c, send, bytes_each, recv, rb.data(), ro.data());
}

void comm_allgatherv_bytes(Ctx& c, const void* send, size_t send_bytes, void* recv, const size_t* recv_bytes,
                           const size_t* recv_off) {
  if (!c.sharded) {
    if (send_bytes && static_cast<uint8_t*>(recv) + recv_off[0] != send)
      NBG_HIP(hipMemcpyAsync(static_cast<uint8_t*>(recv) + recv_off[0], send, send_bytes, hipMemcpyDeviceToDevice,
                             c.stream));
    return;
  }
  impl(c)->allgatherv(c, send, send_bytes, recv, recv_bytes, recv_off);
}

void comm_alltoallv_bytes(Ctx& c, const void* send, const size_t* send_bytes, const size_t* send_off, void* recv,
                          const size_t* recv_bytes, const size_t* recv_off) {
  if (!c.sharded) {
    if (send_bytes[0])
      NBG_HIP(hipMemcpyAsync(static_cast<uint8_t*>(recv) + recv_off[0],
                             static_cast<const uint8_t*>(send) + send_off[0], send_bytes[0],
                             hipMemcpyDeviceToDevice, c.stream));
    return;
  }
  impl(c)->alltoallv(c, send, send_bytes, send_off, recv, recv_bytes, recv_off);
}

void comm_allgatherv2_bytes(Ctx& c, const void* send, size_t send_bytes, void* recv, const size_t* recv_bytes,
                            const size_t* recv_off, const void* send2, size_t bytes2, void* recv2) {
  if (!c.sharded) {
    if (send_bytes && static_cast<uint8_t*>(recv) + recv_off[0] != send)
      NBG_HIP(hipMemcpyAsync(static_cast<uint8_t*>(recv) + recv_off[0], send, send_bytes, hipMemcpyDeviceToDevice,
                             c.stream));
    NBG_HIP(hipMemcpyAsync(recv2, send2, bytes2, hipMemcpyDeviceToDevice, c.stream));
    return;
  }
  impl(c)->allgatherv2(c, send, send_bytes, recv, recv_bytes, recv_off, send2, bytes2, recv2);
}

void comm_allreduce_sum_i64(Ctx& c, int64_t* d_vals, size_t n) {
  if (!c.sharded) return;
  impl(c)->allreduce_sum_i64(c, d_vals, n);
}

}  // namespace nbg
