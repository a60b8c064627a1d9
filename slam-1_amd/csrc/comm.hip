// Collectives of the sharded local BA behind the C ABI:
// RCCL over xGMI, one communicator per rank, one rank per GPU.
//
// The reference has one serial least_squares call (BundleAdjustment.py:397-402);
// the sharded form splits the landmarks by anchor keyframe over the ranks
// (slam355.dist.shard_by_anchor), and one LM iteration is
//   slam_ba_build_system      this rank's partial reduced camera system
//   all-reduce (sum, f64)     the packed system: S blocks + b + g + diag U + cost
//   slam_ba_solve_step        camera solve (every rank), back substitution,
//                             this rank's trial partial sums into prob->small
//   all-reduce (sum, f64)     prob->small (trial |r|^2, predicted decrease)
//   slam_ba_decide            accept / reject, lambda
// slam_ba_step_distributed issues exactly that sequence on one stream, so a C
// caller gets the sharded BA without torch.distributed; the Python layer keeps
// torch.distributed (backend "nccl" = RCCL) as its default and can use this
// communicator instead (slam355.dist.CapiComm).
//
// RCCL is resolved at run time (dlopen / dlsym): the library is linked against
// nothing but the HIP runtime, a process that never calls slam_comm_* never
// loads RCCL, and a process that already has an RCCL exporting the nccl*
// symbols globally uses that one.  SLAM_RCCL_LIB names another library file.
#include "common.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

namespace {

struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
  char why[256] = "";
};

Rccl g_rccl;
std::once_flag g_rccl_once;

template <class F>
bool bind(void* h, const char* name, F* fn) {
  void* s = h ? dlsym(h, name) : dlsym(RTLD_DEFAULT, name);
  *fn = reinterpret_cast<F>(s);
  return s != nullptr;
}

void load_rccl() {
  Rccl& r = g_rccl;
  const char* env = getenv("SLAM_RCCL_LIB");
  void* h = nullptr;
  if (env == nullptr && dlsym(RTLD_DEFAULT, "ncclCommInitRank") != nullptr) {
    h = nullptr;  // an RCCL already in the global scope
  } else {
    const char* names[] = {env, "librccl.so.1", "librccl.so"};
    for (const char* n : names) {
      if (n == nullptr) continue;
      h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
      if (h != nullptr) break;
    }
    if (h == nullptr) {
      snprintf(r.why, sizeof(r.why), "RCCL not loadable (%s)", dlerror());
      return;
    }
  }
  r.ok = bind(h, "ncclGetUniqueId", &r.get_unique_id) && bind(h, "ncclCommInitRank", &r.comm_init_rank) &&
         bind(h, "ncclAllReduce", &r.all_reduce) && bind(h, "ncclCommDestroy", &r.comm_destroy) &&
         bind(h, "ncclGetErrorString", &r.error_string);
  if (!r.ok) snprintf(r.why, sizeof(r.why), "RCCL library lacks an nccl* entry point");
}

int need_rccl() {
  std::call_once(g_rccl_once, load_rccl);
  SLAM_REQUIRE(g_rccl.ok, "slam_comm: %s", g_rccl.why);
  return SLAM_OK;
}

#define SLAM_NCCL(call)                                                                  \
  do {                                                                                  \
    const ncclResult_t r_ = (call);                                                     \
    if (r_ != ncclSuccess) {                                                            \
      ::slam::set_error("%s failed: %s", #call, g_rccl.error_string(r_));               \
      return SLAM_ERR_COMM;                                                             \
    }                                                                                   \
  } while (0)

static_assert(sizeof(ncclUniqueId) == SLAM_COMM_ID_BYTES, "unique id size");

}  // namespace

extern "C" int slam_comm_unique_id(void* h_id) {
  SLAM_REQUIRE(h_id != nullptr, "slam_comm_unique_id: null id buffer");
  if (int rc = need_rccl()) return rc;
  ncclUniqueId id;
  SLAM_NCCL(g_rccl.get_unique_id(&id));
  memcpy(h_id, &id, sizeof(id));
  return SLAM_OK;
}

extern "C" int slam_comm_init(int nranks, int rank, const void* h_id, slam_comm_t* comm) {
  SLAM_REQUIRE(comm != nullptr && h_id != nullptr, "slam_comm_init: null argument");
  SLAM_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "slam_comm_init: rank %d of %d", rank,
               nranks);
  *comm = nullptr;
  if (int rc = need_rccl()) return rc;
  ncclUniqueId id;
  memcpy(&id, h_id, sizeof(id));
  ncclComm_t c = nullptr;
  SLAM_NCCL(g_rccl.comm_init_rank(&c, nranks, id, rank));  // collective over the ranks
  *comm = reinterpret_cast<slam_comm_t>(c);
  return SLAM_OK;
}

extern "C" int slam_comm_destroy(slam_comm_t comm) {
  if (comm == nullptr) return SLAM_OK;
  if (int rc = need_rccl()) return rc;
  SLAM_NCCL(g_rccl.comm_destroy(reinterpret_cast<ncclComm_t>(comm)));
  return SLAM_OK;
}

extern "C" int slam_comm_allreduce_f64(slam_comm_t comm, double* d_buf, long long n, void* stream) {
  SLAM_REQUIRE(comm != nullptr, "slam_comm_allreduce_f64: null communicator");
  SLAM_REQUIRE(n >= 0 && (n == 0 || d_buf != nullptr), "slam_comm_allreduce_f64: bad buffer");
  if (n == 0) return SLAM_OK;
  if (int rc = need_rccl()) return rc;
  SLAM_NCCL(g_rccl.all_reduce(d_buf, d_buf, (size_t)n, ncclFloat64, ncclSum,
                              reinterpret_cast<ncclComm_t>(comm), slam::as_stream(stream)));
  return SLAM_OK;
}

extern "C" int slam_ba_step_distributed(const slam_ba_problem* prob, slam_comm_t comm, void* stream) {
  SLAM_REQUIRE(prob != nullptr && comm != nullptr, "slam_ba_step_distributed: null argument");
  const long long n_sys = slam_ba_sys_len(prob->n_cams, prob->n_blocks);
  SLAM_REQUIRE(n_sys > 0, "slam_ba_step_distributed: bad problem sizes");
  if (int rc = slam_ba_build_system(prob, stream)) return rc;
  if (int rc = slam_comm_allreduce_f64(comm, prob->sys, n_sys, stream)) return rc;
  if (int rc = slam_ba_solve_step(prob, stream)) return rc;
  if (int rc = slam_comm_allreduce_f64(comm, prob->small, 4, stream)) return rc;
  return slam_ba_decide(prob, stream);
}
