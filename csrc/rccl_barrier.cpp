// nos node-atomic commit barrier over RCCL (xGMI).
//
// After the partition agent has applied a plan to every GPU of its node it must not publish the new
// status (the plan-ID commit marker, reference annotations.go:25-28) until every logical device is
// alive and the fabric between them is reachable. One 4-byte ncclAllReduce(sum) over a communicator
// spanning the node's devices is that barrier: each rank contributes 1 if its local apply+verify
// succeeded, so the sum equals nranks iff the whole node committed.
//
// The communicator is created per commit, in a short-lived helper process the partition agent
// spawns (walkai_nos_amd/cmd/gpuhelper.py), and destroyed with it before the next mode flip: a flip
// re-enumerates devices and invalidates every handle, and a process holding a KFD context on the
// GPU is exactly what makes the flip fail with "busy". A 4-byte all-reduce is latency bound (tens of
// microseconds), so link bandwidth (7 x ~153 GB/s xGMI per GPU) is irrelevant here.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {
thread_local std::string g_err;

int nccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return 0;
  g_err = std::string(what) + ": " + ncclGetErrorString(r);
  return int(r) + 1000;
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return int(e);
}

struct Barrier {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  int32_t* dbuf = nullptr;
  int device = 0;
};
}  // namespace

extern "C" {

const char* nos_barrier_last_error() { return g_err.c_str(); }

int nos_barrier_id_size() { return int(sizeof(ncclUniqueId)); }

int nos_barrier_unique_id(char* out, int len) {
  if (len < int(sizeof(ncclUniqueId))) {
    g_err = "buffer too small for ncclUniqueId";
    return -1;
  }
  ncclUniqueId id;
  if (int rc = nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId")) return rc;
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

static void release(Barrier* b) {
  if (b == nullptr) return;
  (void)hipSetDevice(b->device);
  if (b->dbuf) (void)hipFree(b->dbuf);
  if (b->stream) (void)hipStreamDestroy(b->stream);
  delete b;
}

int nos_barrier_init(int nranks, int rank, const char* id_bytes, int device, void** handle) {
  auto* b = new Barrier();
  b->device = device;
  int rc = hip_check(hipSetDevice(device), "hipSetDevice");
  if (!rc) rc = hip_check(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking), "hipStreamCreate");
  if (!rc) rc = hip_check(hipMalloc(&b->dbuf, sizeof(int32_t)), "hipMalloc");
  if (!rc) {
    ncclUniqueId id;
    std::memcpy(&id, id_bytes, sizeof(id));
    rc = nccl_check(ncclCommInitRank(&b->comm, nranks, id, rank), "ncclCommInitRank");
  }
  if (rc) {
    release(b);  // every partially created resource, not just the struct
    return rc;
  }
  *handle = b;
  return 0;
}

// value: this rank's vote (1 = committed). result: the sum over ranks.
int nos_barrier_allreduce(void* handle, int32_t value, int32_t* result) {
  auto* b = static_cast<Barrier*>(handle);
  if (int rc = hip_check(hipSetDevice(b->device), "hipSetDevice")) return rc;
  if (int rc = hip_check(hipMemcpyAsync(b->dbuf, &value, sizeof(value), hipMemcpyHostToDevice, b->stream), "h2d")) return rc;
  if (int rc = nccl_check(ncclAllReduce(b->dbuf, b->dbuf, 1, ncclInt32, ncclSum, b->comm, b->stream), "ncclAllReduce")) return rc;
  if (int rc = hip_check(hipMemcpyAsync(result, b->dbuf, sizeof(int32_t), hipMemcpyDeviceToHost, b->stream), "d2h")) return rc;
  return hip_check(hipStreamSynchronize(b->stream), "hipStreamSynchronize");
}

int nos_barrier_destroy(void* handle) {
  auto* b = static_cast<Barrier*>(handle);
  int rc = 0;
  if (b->comm) rc = nccl_check(ncclCommDestroy(b->comm), "ncclCommDestroy");
  b->comm = nullptr;
  release(b);
  return rc;
}

// Number of HIP devices this process sees (after a compute-partition flip: the partitions). The
// node barrier runs in a freshly spawned helper so that this count, and the HIP context it
// creates, never live in the partition agent itself.
int nos_barrier_device_count() {
  int n = 0;
  if (hip_check(hipGetDeviceCount(&n), "hipGetDeviceCount")) return -1;
  return n;
}

// ---- single-process node barrier: one communicator clique over every local device ------------
// The partition agent is one process per node; ncclCommInitAll gives it one rank per local GPU
// (logical device after the mode flip), and a grouped all-reduce sums the per-device votes.
struct NodeBarrier {
  int n = 0;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;
  std::vector<int32_t*> bufs;
  std::vector<int> devs;
};

static void release_all(NodeBarrier* b) {
  if (b == nullptr) return;
  for (int i = 0; i < b->n; ++i) {
    (void)hipSetDevice(b->devs[i]);
    if (b->bufs[i]) (void)hipFree(b->bufs[i]);
    if (b->streams[i]) (void)hipStreamDestroy(b->streams[i]);
  }
  delete b;
}

int nos_barrier_init_all(int ndev, const int* devlist, void** handle) {
  auto* b = new NodeBarrier();
  b->n = ndev;
  b->devs.assign(devlist, devlist + ndev);
  b->comms.assign(ndev, nullptr);
  b->streams.assign(ndev, nullptr);
  b->bufs.assign(ndev, nullptr);
  int rc = 0;
  for (int i = 0; i < ndev && !rc; ++i) {
    rc = hip_check(hipSetDevice(b->devs[i]), "hipSetDevice");
    if (!rc) rc = hip_check(hipStreamCreateWithFlags(&b->streams[i], hipStreamNonBlocking), "hipStreamCreate");
    if (!rc) rc = hip_check(hipMalloc(&b->bufs[i], sizeof(int32_t)), "hipMalloc");
  }
  if (!rc) rc = nccl_check(ncclCommInitAll(b->comms.data(), ndev, b->devs.data()), "ncclCommInitAll");
  if (rc) {
    for (int i = 0; i < ndev; ++i)
      if (b->comms[i]) (void)ncclCommDestroy(b->comms[i]);
    release_all(b);
    return rc;
  }
  *handle = b;
  return 0;
}

int nos_barrier_allreduce_all(void* handle, const int32_t* votes, int32_t* result) {
  auto* b = static_cast<NodeBarrier*>(handle);
  for (int i = 0; i < b->n; ++i) {
    if (int rc = hip_check(hipSetDevice(b->devs[i]), "hipSetDevice")) return rc;
    if (int rc = hip_check(hipMemcpyAsync(b->bufs[i], &votes[i], sizeof(int32_t), hipMemcpyHostToDevice, b->streams[i]), "h2d")) return rc;
  }
  if (int rc = nccl_check(ncclGroupStart(), "ncclGroupStart")) return rc;
  // every enqueue error is recorded, but the group is always closed: returning from inside an
  // open group leaves the calling thread's group depth at 1, and the next NCCL call of this
  // process would silently join a group that is never launched
  int enq = 0;
  for (int i = 0; i < b->n && !enq; ++i)
    enq = nccl_check(ncclAllReduce(b->bufs[i], b->bufs[i], 1, ncclInt32, ncclSum, b->comms[i], b->streams[i]),
                     "ncclAllReduce");
  std::string enq_err = g_err;
  int end = nccl_check(ncclGroupEnd(), "ncclGroupEnd");
  if (enq) {
    g_err = enq_err;
    return enq;
  }
  if (end) return end;
  for (int i = 0; i < b->n; ++i) {
    if (int rc = hip_check(hipSetDevice(b->devs[i]), "hipSetDevice")) return rc;
    if (int rc = hip_check(hipStreamSynchronize(b->streams[i]), "hipStreamSynchronize")) return rc;
  }
  if (int rc = hip_check(hipSetDevice(b->devs[0]), "hipSetDevice")) return rc;
  return hip_check(hipMemcpy(result, b->bufs[0], sizeof(int32_t), hipMemcpyDeviceToHost), "d2h");
}

int nos_barrier_destroy_all(void* handle) {
  auto* b = static_cast<NodeBarrier*>(handle);
  int rc = 0;
  for (int i = 0; i < b->n; ++i)
    if (b->comms[i]) rc |= nccl_check(ncclCommDestroy(b->comms[i]), "ncclCommDestroy");
  release_all(b);
  return rc;
}

}  // extern "C"
