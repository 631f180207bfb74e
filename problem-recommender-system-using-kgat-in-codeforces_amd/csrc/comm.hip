// (e) The multi-GPU transport behind the C-ABI (kgat_comm_init /
// allreduce / allgather_rows / reduce_scatter_rows): an RCCL communicator over
// xGMI behind an opaque handle.  The reference has no counterpart -- it runs on
// one device (src/model/KGAT/main.py:239) -- these are the collectives of the
// data-parallel replicas (replicas.py) and of the row-sharded propagation ring
// (sharded.py) for hosts that drive the library without torch.distributed.
//
// RCCL is bound at run time (dlopen): the library does not depend on RCCL
// unless a communicator is made, and a host that already carries an RCCL
// (torch ships its own, without a soname) can hand its path to kgat_comm_load
// so the process holds one RCCL instance.  Every call is stream-ordered on the
// caller's stream; the handle owns its ncclComm_t.
#include <dlfcn.h>

#include <cstring>
#include <mutex>

#include <rccl/rccl.h>

#include "common.hpp"

namespace kgat {
namespace {

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

Rccl g_rccl;
std::mutex g_mu;

template <typename F>
bool bind(void* h, const char* name, F& fn) {
  fn = reinterpret_cast<F>(dlsym(h, name));
  return fn != nullptr;
}

int load_locked(const char* path) {
  if (g_rccl.handle != nullptr) return KGAT_OK;
  void* h = dlopen(path != nullptr && path[0] != '\0' ? path : "librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (h == nullptr) return KGAT_ERR_COMM_UNAVAILABLE;
  Rccl r;
  r.handle = h;
  if (!bind(h, "ncclGetUniqueId", r.get_unique_id) || !bind(h, "ncclCommInitRank", r.comm_init_rank) ||
      !bind(h, "ncclCommDestroy", r.comm_destroy) || !bind(h, "ncclAllReduce", r.all_reduce) ||
      !bind(h, "ncclAllGather", r.all_gather) || !bind(h, "ncclReduceScatter", r.reduce_scatter) ||
      !bind(h, "ncclSend", r.send) || !bind(h, "ncclRecv", r.recv) || !bind(h, "ncclGroupStart", r.group_start) ||
      !bind(h, "ncclGroupEnd", r.group_end) || !bind(h, "ncclGetErrorString", r.error_string)) {
    dlclose(h);
    return KGAT_ERR_COMM_UNAVAILABLE;
  }
  g_rccl = r;
  return KGAT_OK;
}

int ensure_loaded() {
  std::lock_guard<std::mutex> lk(g_mu);
  return load_locked(nullptr);
}

inline int status(ncclResult_t r) { return r == ncclSuccess ? KGAT_OK : KGAT_ERR_COMM_BASE + static_cast<int>(r); }

}  // namespace
}  // namespace kgat

struct kgat_comm {
  ncclComm_t comm;
  int32_t rank, world, device;
};

extern "C" int kgat_comm_load(const char* rccl_path) {
  std::lock_guard<std::mutex> lk(kgat::g_mu);
  return kgat::load_locked(rccl_path);
}

extern "C" const char* kgat_comm_error_string(int status) {
  using namespace kgat;
  if (status < KGAT_ERR_COMM_BASE || status >= KGAT_ERR_COMM_BASE + 100 || g_rccl.error_string == nullptr)
    return "kgat: RCCL error";
  return g_rccl.error_string(static_cast<ncclResult_t>(status - KGAT_ERR_COMM_BASE));
}

extern "C" int kgat_comm_unique_id(uint8_t* id) {
  using namespace kgat;
  if (id == nullptr) return KGAT_ERR_INVALID;
  if (int e = ensure_loaded()) return e;
  static_assert(sizeof(ncclUniqueId) == KGAT_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId u;
  if (int e = status(g_rccl.get_unique_id(&u))) return e;
  memcpy(id, &u, sizeof(u));
  return KGAT_OK;
}

extern "C" int kgat_comm_init(int32_t rank, int32_t world, const uint8_t* id, int32_t device, kgat_comm** out) {
  using namespace kgat;
  if (id == nullptr || out == nullptr || world < 1 || rank < 0 || rank >= world || device < 0) return KGAT_ERR_INVALID;
  if (int e = ensure_loaded()) return e;
  // ncclCommInitRank binds the communicator to the current device: switch to `device` for the
  // call and restore the caller's device afterwards (success or not) -- a library call must not
  // change which GPU the calling thread launches on
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return KGAT_ERR_INVALID;
  if (hipSetDevice(device) != hipSuccess) return KGAT_ERR_INVALID;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  const int e = status(g_rccl.comm_init_rank(&c, world, u, rank));
  const bool restored = hipSetDevice(prev) == hipSuccess;
  if (e) return e;
  if (!restored) {
    g_rccl.comm_destroy(c);
    return KGAT_ERR_INVALID;
  }
  *out = new kgat_comm{c, rank, world, device};
  return KGAT_OK;
}

extern "C" int kgat_comm_destroy(kgat_comm* c) {
  using namespace kgat;
  if (c == nullptr) return KGAT_OK;
  const int e = status(g_rccl.comm_destroy(c->comm));
  delete c;
  return e;
}

extern "C" int kgat_comm_rank(const kgat_comm* c, int32_t* rank, int32_t* world) {
  if (c == nullptr || rank == nullptr || world == nullptr) return KGAT_ERR_INVALID;
  *rank = c->rank;
  *world = c->world;
  return KGAT_OK;
}

extern "C" int kgat_comm_allreduce_sum_f32(kgat_comm* c, const float* send, float* recv, int64_t count,
                                           void* stream) {
  using namespace kgat;
  if (c == nullptr || count < 0 || (count > 0 && (send == nullptr || recv == nullptr))) return KGAT_ERR_INVALID;
  if (count == 0) return KGAT_OK;
  return status(g_rccl.all_reduce(send, recv, static_cast<size_t>(count), ncclFloat32, ncclSum, c->comm,
                                  reinterpret_cast<hipStream_t>(stream)));
}

extern "C" int kgat_comm_allgather_rows(kgat_comm* c, const void* send, void* recv, int64_t bytes_per_rank,
                                        void* stream) {
  using namespace kgat;
  if (c == nullptr || bytes_per_rank < 0 || (bytes_per_rank > 0 && (send == nullptr || recv == nullptr)))
    return KGAT_ERR_INVALID;
  if (bytes_per_rank == 0) return KGAT_OK;
  return status(g_rccl.all_gather(send, recv, static_cast<size_t>(bytes_per_rank), ncclUint8, c->comm,
                                  reinterpret_cast<hipStream_t>(stream)));
}

extern "C" int kgat_comm_reduce_scatter_rows_f32(kgat_comm* c, const float* send, float* recv,
                                                 int64_t count_per_rank, void* stream) {
  using namespace kgat;
  if (c == nullptr || count_per_rank < 0 || (count_per_rank > 0 && (send == nullptr || recv == nullptr)))
    return KGAT_ERR_INVALID;
  if (count_per_rank == 0) return KGAT_OK;
  return status(g_rccl.reduce_scatter(send, recv, static_cast<size_t>(count_per_rank), ncclFloat32, ncclSum,
                                      c->comm, reinterpret_cast<hipStream_t>(stream)));
}

extern "C" int kgat_comm_ring_exchange(kgat_comm* c, const void* send, void* recv, int64_t bytes, void* stream) {
  using namespace kgat;
  if (c == nullptr || bytes < 0 || (bytes > 0 && (send == nullptr || recv == nullptr))) return KGAT_ERR_INVALID;
  if (bytes == 0) return KGAT_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int next = (c->rank + 1) % c->world, prev = (c->rank + c->world - 1) % c->world;
  if (int e = status(g_rccl.group_start())) return e;
  const int e1 = status(g_rccl.send(send, static_cast<size_t>(bytes), ncclUint8, next, c->comm, st));
  const int e2 = status(g_rccl.recv(recv, static_cast<size_t>(bytes), ncclUint8, prev, c->comm, st));
  const int e3 = status(g_rccl.group_end());
  return e1 ? e1 : e2 ? e2 : e3;
}

extern "C" int kgat_comm_gather_at(kgat_comm* c, const void* send, void* recv, const int64_t* dst_off,
                                   const int64_t* nbytes, void* stream) {
  using namespace kgat;
  if (c == nullptr || dst_off == nullptr || nbytes == nullptr || recv == nullptr) return KGAT_ERR_INVALID;
  for (int r = 0; r < c->world; ++r)
    if (nbytes[r] < 0 || dst_off[r] < 0) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  char* out = static_cast<char*>(recv);
  const int64_t mine = nbytes[c->rank];
  if (mine > 0 && send == nullptr) return KGAT_ERR_INVALID;
  if (mine > 0 && send != out + dst_off[c->rank] &&
      hipMemcpyAsync(out + dst_off[c->rank], send, static_cast<size_t>(mine), hipMemcpyDeviceToDevice, st) !=
          hipSuccess)
    return KGAT_ERR_INVALID;
  if (c->world == 1) return KGAT_OK;
  if (int e = status(g_rccl.group_start())) return e;
  int err = KGAT_OK;
  for (int p = 0; p < c->world && !err; ++p) {
    if (p == c->rank) continue;
    if (mine > 0) err = status(g_rccl.send(send, static_cast<size_t>(mine), ncclUint8, p, c->comm, st));
    if (!err && nbytes[p] > 0)
      err = status(g_rccl.recv(out + dst_off[p], static_cast<size_t>(nbytes[p]), ncclUint8, p, c->comm, st));
  }
  const int e2 = status(g_rccl.group_end());
  return err ? err : e2;
}

extern "C" int kgat_comm_allgatherv(kgat_comm* c, const void* send, void* recv, const int64_t* offsets, void* stream) {
  using namespace kgat;
  if (c == nullptr || offsets == nullptr || recv == nullptr) return KGAT_ERR_INVALID;
  if (c->world > KGAT_COMM_MAX_WORLD) return KGAT_ERR_INVALID;
  int64_t off[KGAT_COMM_MAX_WORLD], len[KGAT_COMM_MAX_WORLD];
  for (int r = 0; r < c->world; ++r) {
    if (offsets[r + 1] < offsets[r]) return KGAT_ERR_INVALID;
    off[r] = offsets[r];
    len[r] = offsets[r + 1] - offsets[r];
  }
  return kgat_comm_gather_at(c, send, recv, off, len, stream);
}

extern "C" int kgat_comm_alltoallv(kgat_comm* c, const void* send, const int64_t* send_off, void* recv,
                                   const int64_t* recv_off, void* stream) {
  using namespace kgat;
  if (c == nullptr || send_off == nullptr || recv_off == nullptr) return KGAT_ERR_INVALID;
  for (int r = 0; r < c->world; ++r)
    if (send_off[r + 1] < send_off[r] || recv_off[r + 1] < recv_off[r]) return KGAT_ERR_INVALID;
  if ((send_off[c->world] > send_off[0] && send == nullptr) || (recv_off[c->world] > recv_off[0] && recv == nullptr))
    return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const char* in = static_cast<const char*>(send);
  char* out = static_cast<char*>(recv);
  const int64_t own = send_off[c->rank + 1] - send_off[c->rank];
  if (own != recv_off[c->rank + 1] - recv_off[c->rank]) return KGAT_ERR_INVALID;
  if (own > 0 && hipMemcpyAsync(out + recv_off[c->rank], in + send_off[c->rank], static_cast<size_t>(own),
                                hipMemcpyDeviceToDevice, st) != hipSuccess)
    return KGAT_ERR_INVALID;
  if (c->world == 1) return KGAT_OK;
  if (int e = status(g_rccl.group_start())) return e;
  int err = KGAT_OK;
  for (int p = 0; p < c->world && !err; ++p) {
    if (p == c->rank) continue;
    const int64_t sb = send_off[p + 1] - send_off[p], rb = recv_off[p + 1] - recv_off[p];
    if (sb > 0) err = status(g_rccl.send(in + send_off[p], static_cast<size_t>(sb), ncclUint8, p, c->comm, st));
    if (!err && rb > 0) err = status(g_rccl.recv(out + recv_off[p], static_cast<size_t>(rb), ncclUint8, p, c->comm, st));
  }
  const int e2 = status(g_rccl.group_end());
  return err ? err : e2;
}
