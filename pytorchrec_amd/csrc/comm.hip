// RCCL communicator for the row-sharded exchange, behind the C-ABI (include/mrec.h
// "Communicator"): a binding that is not torch -- cgo, JNI, a C++ trainer -- drives
// the sharded step with these calls and the mrec_shard_* kernels alone.
//
// RCCL is opened at run time (dlopen), not linked: libmrec loads and its other
// entry points work where no RCCL is installed, and inside a process that already
// loaded one (PyTorch's) the same copy is reused (RTLD_NOLOAD first), so the
// communicators of torch.distributed and of libmrec share one library.
//
// Every exchange is an equal-split all-to-all (W parts of a fixed size, SURVEY.md
// §8(e)): grouped point-to-point sends/receives on the caller's stream, so the calls
// are stream-ordered and capturable in a HIP graph like torch's.  A graph that
// captured them must be destroyed before mrec_comm_destroy (RCCL waits for it:
// bench.py teardown, tools/destroy_probe.py).
#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <string>

#include <mutex>

#include "common.h"

namespace {

// the subset of rccl.h this file calls (declared here: the header's API, opened at run time)
typedef int rccl_result;  // ncclResult_t, 0 = ncclSuccess
typedef void *rccl_comm;  // ncclComm_t
struct rccl_id {
  char internal[MREC_COMM_ID_BYTES];
};
enum { kRcclInt8 = 0, kRcclInt32 = 2, kRcclFloat32 = 7 };  // ncclDataType_t
enum { kRcclSum = 0 };                                      // ncclRedOp_t

struct Rccl {
  void *h = nullptr;
  rccl_result (*get_unique_id)(rccl_id *) = nullptr;
  rccl_result (*comm_init_rank)(rccl_comm *, int, rccl_id, int) = nullptr;
  rccl_result (*comm_destroy)(rccl_comm) = nullptr;
  rccl_result (*group_start)() = nullptr;
  rccl_result (*group_end)() = nullptr;
  rccl_result (*send)(const void *, size_t, int, int, rccl_comm, hipStream_t) = nullptr;
  rccl_result (*recv)(void *, size_t, int, int, rccl_comm, hipStream_t) = nullptr;
  rccl_result (*all_reduce)(const void *, void *, size_t, int, int, rccl_comm, hipStream_t) = nullptr;
  const char *(*error_string)(rccl_result) = nullptr;
};

Rccl g_rccl;
std::string g_open_error;
std::once_flag g_rccl_once;

// opens RCCL once per process (std::call_once: concurrent first callers, e.g. one
// host thread per device, all wait for the one load and see its result and error)
void open_rccl() {
  const char *env = getenv("MREC_RCCL_LIB");
  const char *names[] = {env, "librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"};
  void *h = nullptr;
  for (const char *n : names)  // a copy already in the process (PyTorch's) first
    if (n && (h = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) break;
  for (const char *n : names)
    if (!h && n) h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    const char *e = dlerror();
    g_open_error = std::string("cannot open RCCL (librccl.so): ") + (e ? e : "?");
    return;
  }
  Rccl r;
  r.h = h;
  bool ok = true;
  auto sym = [&](const char *name) {
    void *p = dlsym(h, name);
    if (!p) ok = false;
    return p;
  };
  r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
  r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
  r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
  r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
  r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
  r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
  r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
  r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
  r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
  if (!ok) {
    g_open_error = "RCCL library lacks a required symbol";
    return;
  }
  g_rccl = r;
}

bool load_rccl() {
  std::call_once(g_rccl_once, open_rccl);
  return g_rccl.h != nullptr;
}

mrec_status rccl_status(rccl_result r, const char *what) {
  if (r == 0) return MREC_OK;
  mrec::set_error(std::string(what) + ": " +
                  (g_rccl.error_string ? g_rccl.error_string(r) : "RCCL error"));
  return MREC_ERCCL;
}

}  // namespace

struct mrec_comm_s {
  rccl_comm comm;
  int rank;
  int world;
};

// equal-split all-to-all of W parts of `count` elements of `dtype` (element bytes `eb`)
static mrec_status a2a(mrec_comm *c, const void *send, void *recv, int64_t count, int dtype,
                       int eb, mrec_stream stream, const char *what) {
  MREC_CHECK_ARG(c != nullptr, "comm is NULL");
  MREC_CHECK_ARG(count >= 0, "negative count");
  MREC_CHECK_ARG(count == 0 || (send && recv), "NULL buffer");
  if (count == 0) return MREC_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const char *sp = static_cast<const char *>(send);
  char *rp = static_cast<char *>(recv);
  const int64_t part = count * eb;
  mrec_status st = rccl_status(g_rccl.group_start(), what);
  if (st != MREC_OK) return st;
  for (int p = 0; p < c->world; ++p) {
    rccl_result r = g_rccl.send(sp + p * part, static_cast<size_t>(count), dtype, p, c->comm, s);
    if (r == 0) r = g_rccl.recv(rp + p * part, static_cast<size_t>(count), dtype, p, c->comm, s);
    if (r != 0) {
      g_rccl.group_end();
      return rccl_status(r, what);
    }
  }
  return rccl_status(g_rccl.group_end(), what);
}

extern "C" {

mrec_status mrec_comm_unique_id(void *id_out) {
  MREC_CHECK_ARG(id_out != nullptr, "id_out is NULL");
  if (!load_rccl()) {
    mrec::set_error(g_open_error);
    return MREC_ERCCL;
  }
  rccl_id id;
  mrec_status st = rccl_status(g_rccl.get_unique_id(&id), "mrec_comm_unique_id");
  if (st == MREC_OK) memcpy(id_out, id.internal, MREC_COMM_ID_BYTES);
  return st;
}

mrec_status mrec_comm_init(const void *unique_id, int32_t rank, int32_t world, mrec_comm **out) {
  MREC_CHECK_ARG(unique_id != nullptr && out != nullptr, "NULL pointer");
  MREC_CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "rank must be in [0, world)");
  *out = nullptr;
  if (!load_rccl()) {
    mrec::set_error(g_open_error);
    return MREC_ERCCL;
  }
  rccl_id id;
  memcpy(id.internal, unique_id, MREC_COMM_ID_BYTES);
  rccl_comm comm = nullptr;
  mrec_status st = rccl_status(g_rccl.comm_init_rank(&comm, world, id, rank), "mrec_comm_init");
  if (st != MREC_OK) return st;
  *out = new mrec_comm_s{comm, rank, world};
  return MREC_OK;
}

mrec_status mrec_comm_destroy(mrec_comm *comm) {
  if (comm == nullptr) return MREC_OK;
  mrec_status st = rccl_status(g_rccl.comm_destroy(comm->comm), "mrec_comm_destroy");
  delete comm;
  return st;
}

int32_t mrec_comm_world(const mrec_comm *comm) { return comm ? comm->world : 0; }
int32_t mrec_comm_rank(const mrec_comm *comm) { return comm ? comm->rank : -1; }

mrec_status mrec_a2a_ids(mrec_comm *comm, const int32_t *send_ids, int32_t *recv_ids,
                         int64_t per_peer, mrec_stream stream) {
  return a2a(comm, send_ids, recv_ids, per_peer, kRcclInt32, 4, stream, "mrec_a2a_ids");
}

mrec_status mrec_a2a_rows_fwd(mrec_comm *comm, const void *send_rows, void *recv_rows,
                              int64_t bytes_per_peer, mrec_stream stream) {
  MREC_CHECK_ARG(bytes_per_peer % 16 == 0, "rows are whole 16-B units");
  return a2a(comm, send_rows, recv_rows, bytes_per_peer, kRcclInt8, 1, stream,
             "mrec_a2a_rows_fwd");
}

mrec_status mrec_a2a_rows_bwd(mrec_comm *comm, const float *send_grads, float *recv_grads,
                              int64_t floats_per_peer, mrec_stream stream) {
  return a2a(comm, send_grads, recv_grads, floats_per_peer, kRcclFloat32, 4, stream,
             "mrec_a2a_rows_bwd");
}

mrec_status mrec_allreduce_sum_f32(mrec_comm *comm, float *buf, int64_t n, mrec_stream stream) {
  MREC_CHECK_ARG(comm != nullptr, "comm is NULL");
  MREC_CHECK_ARG(n >= 0 && (n == 0 || buf), "bad buffer");
  if (n == 0) return MREC_OK;
  return rccl_status(g_rccl.all_reduce(buf, buf, static_cast<size_t>(n), kRcclFloat32, kRcclSum,
                                       comm->comm, static_cast<hipStream_t>(stream)),
                     "mrec_allreduce_sum_f32");
}

}  // extern "C"
