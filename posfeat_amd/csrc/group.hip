// group.hip -- cross-rank reduction of small fp64 statistic vectors for
// SyncBatchNorm semantics in the train-mode backbone (bbtrain.hip).
//
// Replaces: torch.nn.SyncBatchNorm.convert_sync_batchnorm of the reference's
//   PoSFeat.set_parallel (networks/PoSFeat_model.py:48-55): under DDP every
//   BatchNorm of the backbone computes its batch statistics over the union of
//   the ranks' batches (forward: sum y, sum y^2; backward: sum g, sum g x^).
//
// One exchange = an in-place sum over ranks of `n` doubles on the caller's
// stream.  Three implementations behind one handle:
//   * RCCL: ncclAllReduce(fp64, sum) on a communicator created from a unique
//     id the host broadcasts (torch.distributed on the host side).  librccl is
//     resolved at run time (dlopen; the copy torch already loaded first), so
//     this library has no link-time RCCL dependency.
//   * host: a process group without RCCL (gloo; e.g. ranks sharing one
//     device, where RCCL refuses a second rank on the same GPU): the vector
//     goes to pinned host memory, a caller callback sums it over the ranks
//     (torch.distributed.all_reduce in parallel.SyncBNGroup), and back.
//   * local: N "ranks" that are threads of one process on one device (tests:
//     two half-batch ranks against one full-batch run on a one-GPU box).  Rank
//     r copies its vector into slot r of a shared device buffer; after a host
//     barrier every rank sums the slots in rank order (deterministic); a second
//     barrier frees the slots for the next exchange.
#include <dlfcn.h>

#include <condition_variable>
#include <cstring>
#include <mutex>

#include "common.h"
#include "group.h"

namespace {

// minimal RCCL ABI (rccl.h: ncclUniqueId = 128 bytes, ncclFloat64 = 8, ncclSum = 0)
struct UniqueId {
  char internal[128];
};
typedef void* Comm;
typedef int (*GetUniqueIdFn)(UniqueId*);
typedef int (*CommInitRankFn)(Comm*, int, UniqueId, int);
typedef int (*AllReduceFn)(const void*, void*, size_t, int, int, Comm, hipStream_t);
typedef int (*CommDestroyFn)(Comm);

struct Rccl {
  GetUniqueIdFn get_id = nullptr;
  CommInitRankFn init = nullptr;
  AllReduceFn allreduce = nullptr;
  CommDestroyFn destroy = nullptr;
  bool ok = false;
};

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.get_id = reinterpret_cast<GetUniqueIdFn>(dlsym(h, "ncclGetUniqueId"));
    x.init = reinterpret_cast<CommInitRankFn>(dlsym(h, "ncclCommInitRank"));
    x.allreduce = reinterpret_cast<AllReduceFn>(dlsym(h, "ncclAllReduce"));
    x.destroy = reinterpret_cast<CommDestroyFn>(dlsym(h, "ncclCommDestroy"));
    x.ok = x.get_id && x.init && x.allreduce && x.destroy;
    return x;
  }();
  return r;
}

// sum of the world slots (rank order) into out
__global__ void slot_sum_kernel(const double* __restrict__ slots, int world, int stride, int n,
                                double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int r = 0; r < world; ++r) s += slots[(size_t)r * stride + i];
  out[i] = s;
}

}  // namespace

struct posfeat_local_group {
  int world = 0;
  int stride = 0;  // doubles per slot
  double* slots = nullptr;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long long gen = 0;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const long long g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

struct posfeat_group {
  int world = 1, rank = 0;
  Comm comm = nullptr;                     // RCCL
  posfeat_local_group* local = nullptr;    // local emulation
  posfeat_host_allreduce_fn host = nullptr;  // host transport (gloo process groups)
  void* user = nullptr;
  double* hbuf = nullptr;  // pinned staging of the host transport
  int hcap = 0;
};

int pf_group_world(const posfeat_group* g) { return g ? g->world : 1; }

int pf_group_allreduce(posfeat_group* g, double* buf, int n, hipStream_t st) {
  if (!g || g->world == 1) return POSFEAT_OK;
  if (g->comm) {
    const int r = rccl().allreduce(buf, buf, (size_t)n, 8 /*fp64*/, 0 /*sum*/, g->comm, st);
    return r == 0 ? POSFEAT_OK : POSFEAT_E_HIP;
  }
  if (g->host) {
    if (n > g->hcap) {
      if (g->hbuf) (void)hipHostFree(g->hbuf);
      g->hbuf = nullptr;
      g->hcap = 0;
      if (hipHostMalloc(reinterpret_cast<void**>(&g->hbuf), (size_t)n * sizeof(double), 0) !=
          hipSuccess)
        return POSFEAT_E_HIP;
      g->hcap = n;
    }
    if (hipMemcpyAsync(g->hbuf, buf, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return POSFEAT_E_HIP;
    if (g->host(g->hbuf, n, g->user) != 0) return POSFEAT_E_INVALID;
    if (hipMemcpyAsync(buf, g->hbuf, (size_t)n * sizeof(double), hipMemcpyHostToDevice, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return POSFEAT_E_HIP;
    return POSFEAT_OK;
  }
  posfeat_local_group* L = g->local;
  if (n > L->stride) return POSFEAT_E_INVALID;
  if (hipMemcpyAsync(L->slots + (size_t)g->rank * L->stride, buf, n * sizeof(double),
                     hipMemcpyDeviceToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return POSFEAT_E_HIP;
  L->barrier();
  hipLaunchKernelGGL(slot_sum_kernel, dim3((n + 255) / 256), dim3(256), 0, st, L->slots, L->world,
                     L->stride, n, buf);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
    return POSFEAT_E_HIP;
  L->barrier();
  return POSFEAT_OK;
}

extern "C" int posfeat_group_unique_id(void* out128) {
  if (!out128) return POSFEAT_E_INVALID;
  if (!rccl().ok) return POSFEAT_E_UNSUPPORTED;
  UniqueId id;
  if (rccl().get_id(&id) != 0) return POSFEAT_E_HIP;
  memcpy(out128, id.internal, sizeof id.internal);
  return POSFEAT_OK;
}

extern "C" int posfeat_group_create_rccl(int world, int rank, const void* id128,
                                         posfeat_group** out) {
  if (!out || !id128 || world < 1 || rank < 0 || rank >= world) return POSFEAT_E_INVALID;
  if (!rccl().ok) return POSFEAT_E_UNSUPPORTED;
  UniqueId id;
  memcpy(id.internal, id128, sizeof id.internal);
  Comm c = nullptr;
  if (rccl().init(&c, world, id, rank) != 0) return POSFEAT_E_HIP;
  posfeat_group* g = new posfeat_group();
  g->world = world;
  g->rank = rank;
  g->comm = c;
  *out = g;
  return POSFEAT_OK;
}

extern "C" int posfeat_local_group_create(int world, int max_doubles, posfeat_local_group** out) {
  if (!out || world < 1 || max_doubles < 1) return POSFEAT_E_INVALID;
  posfeat_local_group* L = new posfeat_local_group();
  L->world = world;
  L->stride = (max_doubles + 31) / 32 * 32;
  if (hipMalloc(&L->slots, (size_t)world * L->stride * sizeof(double)) != hipSuccess) {
    delete L;
    return POSFEAT_E_HIP;
  }
  *out = L;
  return POSFEAT_OK;
}

extern "C" int posfeat_group_create_local(posfeat_local_group* L, int rank, posfeat_group** out) {
  if (!L || !out || rank < 0 || rank >= L->world) return POSFEAT_E_INVALID;
  posfeat_group* g = new posfeat_group();
  g->world = L->world;
  g->rank = rank;
  g->local = L;
  *out = g;
  return POSFEAT_OK;
}

extern "C" int posfeat_group_create_host(int world, int rank, posfeat_host_allreduce_fn allreduce,
                                         void* user, posfeat_group** out) {
  if (!out || !allreduce || world < 1 || rank < 0 || rank >= world) return POSFEAT_E_INVALID;
  posfeat_group* g = new posfeat_group();
  g->world = world;
  g->rank = rank;
  g->host = allreduce;
  g->user = user;
  *out = g;
  return POSFEAT_OK;
}

extern "C" void posfeat_group_destroy(posfeat_group* g) {
  if (!g) return;
  if (g->comm && rccl().ok) (void)rccl().destroy(g->comm);
  if (g->hbuf) (void)hipHostFree(g->hbuf);
  delete g;
}

extern "C" void posfeat_local_group_destroy(posfeat_local_group* L) {
  if (!L) return;
  if (L->slots) (void)hipFree(L->slots);
  delete L;
}
