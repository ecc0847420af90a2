// Peer-memory one-shot all-reduce over HIP IPC (latency path for small
// collectives), an opt-in data plane (NDP_COMM=ipc, parallel/comm.py).
//
// The reference's collectives (ddp_powersgd_guide_cifar10/reducer.py:126,132,145) are a few
// 0.1-1 MB all-reduces per step: latency-bound.  Here every rank owns one symmetric device
// buffer (data + flag words), exports it with hipIpcGetMemHandle, exchanges the handles
// through the c10d store and maps every peer's buffer with hipIpcOpenMemHandle (dmabuf IPC:
// HSA_ENABLE_IPC_MODE_LEGACY=0).  One kernel per collective, no host synchronisation,
// hipGraph-capturable:
//   workgroup w owns the fixed 16-KB chunk w of the buffer (the chunk -> workgroup mapping
//   never changes, so each workgroup's flags order only its own chunk, and no workgroup
//   waits for another workgroup of its own kernel: no co-residency assumption);
//   with e = this chunk's use count (a device counter, so captured graphs replay):
//     1. wait until every peer has finished reading my chunk w of use e-1 (done flags);
//     2. copy my input chunk into my buffer, release (system scope), write `ready = e` into
//        every peer's flag array;
//     3. wait for every peer's ready flag, acquire, and sum the N chunks in rank order
//        0..N-1 — every rank performs the identical fp32 additions, so the results are
//        bitwise identical across ranks (replica consistency);
//     4. write `done = e` into every peer's flag array.
// Spins are wall-clock bounded (s_memrealtime): a timeout sets a sticky error word and the
// workgroup returns at once (no staging, no sum, no flag writes), later collectives skip,
// and the host check (Communicator.check) fails the run on every rank — never a hang.
// The buffer (data + flags) is allocated UNCACHED (hipDeviceMallocUncached): flags written
// by peers and data a peer rewrites between uses must never be served from a stale cache
// line on the reading side.  If the allocator or IPC export refuses uncached memory the
// buffer falls back to plain hipMalloc and `uncached` is false; then the Python data plane
// only pairs ranks that share one device (parallel/comm.py IpcDataPlane).  Exercised so far
// between processes sharing one GPU (tests/test_ipc_gpu.py); the xGMI case is untested.
// all_reduce_many packs a list of tensors into ONE launch: chunk w covers floats
// [w*4096, (w+1)*4096) of the tensors' concatenation (a segment table in the arguments).
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <ATen/ATen.h>

#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace {

constexpr int kIpcMaxRanks = 16;
constexpr int kIpcChunk = 4096;  // floats per workgroup chunk (16 KB)
constexpr int kIpcThreads = 256;

#define NDP_IPC_CHECK(expr)                                                                \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    TORCH_CHECK(_e == hipSuccess, "HIP error in ", #expr, ": ", hipGetErrorString(_e));     \
  } while (0)

constexpr int kIpcMaxSegs = 48;  // tensors per launch (kernel-argument table)

struct IpcArgs {
  float* data[kIpcMaxRanks];        // every rank's buffer, mapped into this process
  unsigned* ready[kIpcMaxRanks];    // rank j's ready flags [src rank][chunk]
  unsigned* done[kIpcMaxRanks];     // rank j's done flags  [src rank][chunk]
  unsigned* poison[kIpcMaxRanks];   // rank j's "a peer timed out" word
  float* seg[kIpcMaxSegs];          // in/out tensors (or tensor pieces) of this launch
  int64_t end[kIpcMaxSegs];         // prefix sums of their lengths (buffer offsets)
  int nseg;
  int64_t n;                        // floats in this launch = end[nseg - 1]
  unsigned* ctr;                    // per-chunk use counters (local)
  unsigned* err;                    // sticky error word (local)
  uint64_t max_ticks;               // spin bound, 100 MHz ticks
  float scale;                      // 1 (sum) or 1/N (avg)
  int rank, nranks, gmax;
};

__device__ __forceinline__ bool spin_until(const unsigned* p, unsigned want, unsigned* err, uint64_t max_ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((int)(__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - want) < 0) {
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) {
      __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}

// a wait of this rank timed out: tell every peer (their next collective skips and their host
// check fails too, instead of a peer silently reading half-published chunks)
__device__ __forceinline__ void poison_peers(const IpcArgs& a) {
  for (int j = 0; j < a.nranks; ++j)
    __hip_atomic_fetch_or(a.poison[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// buffer offset i (< a.n) -> address inside the launch's tensors; `k` is the caller's
// running segment index (offsets only grow within a thread's loop)
__device__ __forceinline__ float* seg_addr(const IpcArgs& a, int64_t i, int& k) {
  while (i >= a.end[k]) ++k;
  return a.seg[k] + (i - (k ? a.end[k - 1] : 0));
}

__global__ __launch_bounds__(kIpcThreads) void ipc_allreduce_kernel(IpcArgs a) {
  __shared__ unsigned s_e;
  __shared__ int s_skip;
  __shared__ int s_fail;
  const int w = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    s_e = a.ctr[w] + 1u;
    s_skip = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
             __hip_atomic_load(a.poison[a.rank], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
    s_fail = 0;
  }
  __syncthreads();
  if (s_skip) return;  // sticky error: the host check reports it
  const unsigned e = s_e;
  const int R = a.rank, N = a.nranks;
  const int64_t base = (int64_t)w * kIpcChunk;
  const int cnt = (int)min((int64_t)kIpcChunk, a.n - base);

  // 1. peers are done reading my chunk w of the previous use
  if (tid < N && tid != R && e > 1u && !spin_until(a.done[R] + tid * a.gmax + w, e - 1u, a.err, a.max_ticks)) {
    s_fail = 1;
    poison_peers(a);
  }
  __syncthreads();
  if (s_fail) return;  // a peer may still read the old chunk: do not overwrite it
  // 2. stage my contribution, publish it
  float* mine = a.data[R] + base;
  int k = 0;
  for (int i = tid; i < cnt; i += kIpcThreads) mine[i] = *seg_addr(a, base + i, k);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // every wave: its stores reach memory (system scope)
  __syncthreads();
  if (tid < N) __hip_atomic_store(a.ready[tid] + R * a.gmax + w, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. every contribution is there: fixed-order sum
  if (tid < N && !spin_until(a.ready[R] + tid * a.gmax + w, e, a.err, a.max_ticks)) {
    s_fail = 1;
    poison_peers(a);
  }
  __syncthreads();
  if (s_fail) return;  // partial data: leave the caller's tensor and every flag untouched
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  k = 0;
  for (int i = tid; i < cnt; i += kIpcThreads) {
    float acc = a.data[0][base + i];
    for (int j = 1; j < N; ++j) acc += a.data[j][base + i];
    *seg_addr(a, base + i, k) = a.scale == 1.f ? acc : acc * a.scale;
  }
  __syncthreads();
  // 4. I am done reading everyone's chunk w
  if (tid < N) __hip_atomic_store(a.done[tid] + R * a.gmax + w, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid == 0) a.ctr[w] = e;
}

class IpcComm {
 public:
  IpcComm(int rank, int nranks, int device, int64_t capacity_bytes)
      : rank_(rank), nranks_(nranks), device_(device) {
    TORCH_CHECK(nranks >= 1 && nranks <= kIpcMaxRanks && rank >= 0 && rank < nranks, "IpcComm: bad rank/nranks");
    gmax_ = (int)std::max<int64_t>(1, capacity_bytes / (kIpcChunk * (int64_t)sizeof(float)));
    cap_floats_ = (int64_t)gmax_ * kIpcChunk;
    const size_t flags = (2 * (size_t)kIpcMaxRanks * gmax_ + 1) * sizeof(unsigned);  // ready, done, poison
    bytes_ = cap_floats_ * sizeof(float) + flags;
    NDP_IPC_CHECK(hipSetDevice(device));
    // uncached first (see the header); plain device memory if either step refuses it
    if (hipExtMallocWithFlags(&base_, bytes_, hipDeviceMallocUncached) == hipSuccess) {
      hipIpcMemHandle_t h;
      if (hipIpcGetMemHandle(&h, base_) == hipSuccess) {
        uncached_ = true;
      } else {
        (void)hipFree(base_);
        base_ = nullptr;
      }
    }
    (void)hipGetLastError();  // clear a refused attempt
    if (base_ == nullptr) NDP_IPC_CHECK(hipMalloc(&base_, bytes_));
    NDP_IPC_CHECK(hipMemset(base_, 0, bytes_));
    NDP_IPC_CHECK(hipMalloc(&local_, (gmax_ + 1) * sizeof(unsigned)));
    NDP_IPC_CHECK(hipMemset(local_, 0, (gmax_ + 1) * sizeof(unsigned)));
    NDP_IPC_CHECK(hipDeviceSynchronize());  // zeroed before any peer can map it
    peers_.assign(nranks, nullptr);
    peers_[rank] = base_;
    const char* t = std::getenv("NDP_FLAG_WAIT_US");
    timeout_us_ = t ? std::atoll(t) : 30000000LL;
  }
  ~IpcComm() = default;  // released by destroy() (captured graphs may still reference the buffers)

  std::string handle() const {
    hipIpcMemHandle_t h;
    NDP_IPC_CHECK(hipIpcGetMemHandle(&h, base_));
    return std::string(h.reserved, HIP_IPC_HANDLE_SIZE);
  }

  void open(const std::vector<std::string>& handles) {
    TORCH_CHECK((int)handles.size() == nranks_, "IpcComm.open: one handle per rank");
    NDP_IPC_CHECK(hipSetDevice(device_));
    for (int j = 0; j < nranks_; ++j) {
      if (j == rank_) continue;
      TORCH_CHECK(handles[j].size() == HIP_IPC_HANDLE_SIZE, "IpcComm.open: bad handle size");
      hipIpcMemHandle_t h;
      std::memcpy(h.reserved, handles[j].data(), HIP_IPC_HANDLE_SIZE);
      void* p = nullptr;
      NDP_IPC_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      peers_[j] = p;
    }
    opened_ = true;
  }

  void all_reduce(at::Tensor t, const std::string& op, int64_t stream) { all_reduce_many({t}, op, stream); }

  // every tensor of the list in as few launches as the buffer capacity and the segment
  // table allow (one for the PowerSGD payloads)
  void all_reduce_many(const std::vector<at::Tensor>& ts, const std::string& op, int64_t stream) {
    TORCH_CHECK(opened_, "IpcComm: open() the peer handles first");
    TORCH_CHECK(op == "sum" || op == "avg", "IpcComm: sum / avg only");
    for (const auto& t : ts)
      TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kFloat &&
                      t.get_device() == device_,
                  "IpcComm: contiguous float32 tensors on the communicator's device");
    hipStream_t s = stream == 0 ? at::hip::getCurrentHIPStream().stream() : reinterpret_cast<hipStream_t>(stream);
    IpcArgs a{};
    for (int j = 0; j < nranks_; ++j) {
      char* b = static_cast<char*>(peers_[j]);
      a.data[j] = reinterpret_cast<float*>(b);
      a.ready[j] = reinterpret_cast<unsigned*>(b + cap_floats_ * sizeof(float));
      a.done[j] = a.ready[j] + (size_t)kIpcMaxRanks * gmax_;
      a.poison[j] = a.done[j] + (size_t)kIpcMaxRanks * gmax_;
    }
    a.ctr = static_cast<unsigned*>(local_);
    a.err = a.ctr + gmax_;
    a.max_ticks = (uint64_t)(timeout_us_ > 0 ? timeout_us_ : 0) * 100u;
    a.scale = op == "avg" ? 1.f / nranks_ : 1.f;
    a.rank = rank_;
    a.nranks = nranks_;
    a.gmax = gmax_;
    auto flush = [&]() {
      if (a.nseg == 0) return;
      a.n = a.end[a.nseg - 1];
      const int g = (int)((a.n + kIpcChunk - 1) / kIpcChunk);
      hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(g), dim3(kIpcThreads), 0, s, a);
      a.nseg = 0;
      ++launches_;
    };
    for (const auto& t : ts) {
      float* p = t.data_ptr<float>();
      int64_t left = t.numel(), off = 0;
      while (left > 0) {  // a tensor may straddle launches (buffer capacity)
        const int64_t used = a.nseg ? a.end[a.nseg - 1] : 0;
        if (used == cap_floats_ || a.nseg == kIpcMaxSegs) {
          flush();
          continue;
        }
        const int64_t take = std::min<int64_t>(left, cap_floats_ - (a.nseg ? a.end[a.nseg - 1] : 0));
        a.seg[a.nseg] = p + off;
        a.end[a.nseg] = (a.nseg ? a.end[a.nseg - 1] : 0) + take;
        ++a.nseg;
        off += take;
        left -= take;
      }
    }
    flush();
    NDP_IPC_CHECK(hipGetLastError());
  }

  // PCI bus id of the communicator's device (peers compare them: same device or not)
  std::string bus_id() const {
    char buf[64] = {0};
    NDP_IPC_CHECK(hipDeviceGetPCIBusId(buf, sizeof(buf), device_));
    return std::string(buf);
  }

  // host-synchronising: 0, or 1 = a wait of this rank timed out, 2 = a peer's did
  int64_t error() const {
    unsigned v = 0, pv = 0;
    NDP_IPC_CHECK(hipMemcpy(&v, static_cast<unsigned*>(local_) + gmax_, sizeof(unsigned), hipMemcpyDeviceToHost));
    const unsigned* poison = reinterpret_cast<const unsigned*>(static_cast<char*>(base_) + cap_floats_ * sizeof(float)) +
                             2 * (size_t)kIpcMaxRanks * gmax_;
    NDP_IPC_CHECK(hipMemcpy(&pv, poison, sizeof(unsigned), hipMemcpyDeviceToHost));
    return (v ? 1 : 0) | (pv ? 2 : 0);
  }
  void check() const {
    const int64_t e = error();
    TORCH_CHECK(e == 0, "IPC all-reduce: ", (e & 1) ? "a peer wait of this rank" : "a peer's wait",
                " timed out after ", timeout_us_ / 1e6, " s (a stalled or diverged rank); the results since are invalid");
  }
  void destroy() {
    if (base_ == nullptr) return;
    for (int j = 0; j < nranks_; ++j)
      if (j != rank_ && peers_[j] != nullptr) (void)hipIpcCloseMemHandle(peers_[j]);
    (void)hipFree(base_);
    (void)hipFree(local_);
    base_ = local_ = nullptr;
    opened_ = false;
  }
  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  int device() const { return device_; }
  int64_t capacity() const { return cap_floats_ * sizeof(float); }
  bool alive() const { return base_ != nullptr; }
  bool uncached() const { return uncached_; }
  int64_t launches() const { return launches_; }

 private:
  int rank_, nranks_, device_;
  int gmax_ = 0;
  int64_t cap_floats_ = 0;
  size_t bytes_ = 0;
  int64_t timeout_us_ = 0;
  void* base_ = nullptr;
  void* local_ = nullptr;
  bool opened_ = false;
  bool uncached_ = false;
  int64_t launches_ = 0;
  std::vector<void*> peers_;
};

}  // namespace

// C++ surface for the pybind11 registration in bindings.cpp (pybind11 stays out of the
// hipcc-compiled translation units: its inline internals compiled by two compilers in one
// module corrupted the registry at import)
namespace ndp {
void* ipc_new(int rank, int nranks, int device, int64_t capacity_bytes) {
  return new IpcComm(rank, nranks, device, capacity_bytes);
}
void ipc_delete(void* c) { delete static_cast<IpcComm*>(c); }
std::string ipc_handle(void* c) { return static_cast<IpcComm*>(c)->handle(); }
void ipc_open(void* c, const std::vector<std::string>& h) { static_cast<IpcComm*>(c)->open(h); }
void ipc_all_reduce_many(void* c, const std::vector<at::Tensor>& ts, const std::string& op, int64_t stream) {
  static_cast<IpcComm*>(c)->all_reduce_many(ts, op, stream);
}
int64_t ipc_error(void* c) { return static_cast<IpcComm*>(c)->error(); }
void ipc_check(void* c) { static_cast<IpcComm*>(c)->check(); }
void ipc_destroy(void* c) { static_cast<IpcComm*>(c)->destroy(); }
std::string ipc_bus_id(void* c) { return static_cast<IpcComm*>(c)->bus_id(); }
int64_t ipc_info(void* c, int what) {
  const IpcComm* p = static_cast<IpcComm*>(c);
  switch (what) {
    case 0: return p->rank();
    case 1: return p->nranks();
    case 2: return p->device();
    case 3: return p->capacity();
    case 4: return p->alive() ? 1 : 0;
    case 5: return p->uncached() ? 1 : 0;
    default: return p->launches();
  }
}
}  // namespace ndp
