// Native RCCL communicator on framework-owned HIP streams.
//
// The reference drives every collective through c10d (ProcessGroupNCCL):
//   all_reduce(P)              ddp_powersgd_guide_cifar10/reducer.py:126
//   all_reduce(rank-1, async)  reducer.py:132 -> tensor_buffer.py:48
//   all_reduce(Q)              reducer.py:145
//   per-parameter all_reduce   ddp_guide_cifar10/ddp_init.py:61
// Here c10d only bootstraps: rank 0 creates an ncclUniqueId, the Python layer passes its
// 128 bytes through the c10d store, and every rank calls ncclCommInitRank itself.  The
// communicator then enqueues RCCL kernels directly on the caller's current HIP stream —
// in practice the framework-owned high-priority SideStream below, ordered against the
// compute stream with hipEvents, so bucket / PowerSGD-group collectives run while
// backward is still producing gradients (eagerly, or as comm graphs launched between the
// segments of a captured step, utils/graph.py).
// ncclGroupStart/End fuse several collectives into one launch (e.g. the last PowerSGD
// P-group and the rank-1 buffer).  No host synchronisation anywhere; RCCL errors are
// polled with ncclCommGetAsyncError (check()).
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

namespace {

#define NDP_NCCL_CHECK(expr)                                                           \
  do {                                                                                 \
    ncclResult_t _r = (expr);                                                          \
    TORCH_CHECK(_r == ncclSuccess, "RCCL error in ", #expr, ": ", ncclGetErrorString(_r)); \
  } while (0)

#define NDP_HIP_CHECK(expr)                                                             \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    TORCH_CHECK(_e == hipSuccess, "HIP error in ", #expr, ": ", hipGetErrorString(_e)); \
  } while (0)

ncclDataType_t nccl_dtype(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kFloat32: return ncclFloat32;
    case torch::kFloat64: return ncclFloat64;
    case torch::kFloat16: return ncclFloat16;
    case torch::kBFloat16: return ncclBfloat16;
    case torch::kInt32: return ncclInt32;
    case torch::kInt64: return ncclInt64;
    case torch::kUInt8: return ncclUint8;
    case torch::kInt8: return ncclInt8;
    default: TORCH_CHECK(false, "RcclComm: unsupported dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

ncclRedOp_t nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "RcclComm: unknown reduce op ", op);
  return ncclSum;
}

py::bytes unique_id() {
  ncclUniqueId id;
  NDP_NCCL_CHECK(ncclGetUniqueId(&id));
  return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

int rccl_version() {
  int v = 0;
  NDP_NCCL_CHECK(ncclGetVersion(&v));
  return v;
}

class RcclComm {
 public:
  RcclComm(const std::string& uid, int nranks, int rank, int device) : nranks_(nranks), rank_(rank), device_(device) {
    TORCH_CHECK(uid.size() == NCCL_UNIQUE_ID_BYTES, "RcclComm: unique id must be ", NCCL_UNIQUE_ID_BYTES, " bytes");
    TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "RcclComm: bad rank/nranks");
    ncclUniqueId id;
    std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
    NDP_HIP_CHECK(hipSetDevice(device));
    NDP_NCCL_CHECK(ncclCommInitRank(&comm_, nranks, id, rank));
  }

  // No ncclCommDestroy in the destructor: at interpreter shutdown Python frees objects in
  // no particular order, and a captured hipGraph that still holds RCCL kernels of this
  // communicator must not outlive it.  destroy() / abort() release it explicitly
  // (Communicator.close() does so when no graph captured its collectives).
  ~RcclComm() = default;

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  int device() const { return device_; }

  // ---- collectives: enqueue on `stream` (0 = the caller's current stream) -----------
  void all_reduce(torch::Tensor t, const std::string& op, int64_t stream) {
    check_tensor(t);
    NDP_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), nccl_dtype(t), nccl_op(op), comm(),
                                 pick(stream)));
  }

  // several in-place all-reduces fused into one RCCL launch (ncclGroupStart/End)
  void all_reduce_many(const std::vector<torch::Tensor>& ts, const std::string& op, int64_t stream) {
    for (const auto& t : ts) check_tensor(t);
    const hipStream_t s = pick(stream);
    const ncclRedOp_t o = nccl_op(op);
    NDP_NCCL_CHECK(ncclGroupStart());
    for (const auto& t : ts)
      NDP_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), nccl_dtype(t), o, comm(), s));
    NDP_NCCL_CHECK(ncclGroupEnd());
  }

  void broadcast(torch::Tensor t, int root, int64_t stream) {
    check_tensor(t);
    NDP_NCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), nccl_dtype(t), root, comm(),
                                 pick(stream)));
  }

  // out: nranks * in.numel() elements, rank-major
  void all_gather(torch::Tensor out, torch::Tensor in, int64_t stream) {
    check_tensor(out);
    check_tensor(in);
    TORCH_CHECK(out.numel() == in.numel() * nranks_ && out.scalar_type() == in.scalar_type(),
                "all_gather: out must hold nranks * in.numel() elements of the same dtype");
    NDP_NCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), nccl_dtype(in), comm(),
                                 pick(stream)));
  }

  // in: nranks * out.numel() elements; out = this rank's reduced shard
  void reduce_scatter(torch::Tensor out, torch::Tensor in, const std::string& op, int64_t stream) {
    check_tensor(out);
    check_tensor(in);
    TORCH_CHECK(in.numel() == out.numel() * nranks_ && out.scalar_type() == in.scalar_type(),
                "reduce_scatter: in must hold nranks * out.numel() elements of the same dtype");
    NDP_NCCL_CHECK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), (size_t)out.numel(), nccl_dtype(in), nccl_op(op),
                                     comm(), pick(stream)));
  }

  // raises if RCCL reported an asynchronous error (peer failure, timeout, ...)
  void check() {
    if (comm_ == nullptr) return;
    ncclResult_t err = ncclSuccess;
    NDP_NCCL_CHECK(ncclCommGetAsyncError(comm_, &err));
    TORCH_CHECK(err == ncclSuccess || err == ncclInProgress, "RCCL async error: ", ncclGetErrorString(err));
  }

  void abort() { release(true); }
  void destroy() { release(false); }
  bool alive() const { return comm_ != nullptr; }

 private:
  ncclComm_t comm() const {
    TORCH_CHECK(comm_ != nullptr, "RcclComm used after destroy()/abort()");
    return comm_;
  }
  hipStream_t pick(int64_t s) const {
    return s == 0 ? at::hip::getCurrentHIPStream().stream() : reinterpret_cast<hipStream_t>(s);
  }
  void check_tensor(const torch::Tensor& t) const {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RcclComm: tensors must be contiguous device tensors");
    TORCH_CHECK(t.get_device() == device_, "RcclComm: tensor on device ", t.get_device(), ", communicator on ",
                device_);
  }
  void release(bool abort) {
    if (comm_ != nullptr) {
      if (abort) (void)ncclCommAbort(comm_);
      else (void)ncclCommDestroy(comm_);
      comm_ = nullptr;
    }
  }

  ncclComm_t comm_ = nullptr;
  int nranks_, rank_, device_;
};

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  NDP_HIP_CHECK(hipStreamIsCapturing(s, &st));
  return st == hipStreamCaptureStatusActive;
}

hipStream_t cur() { return at::hip::getCurrentHIPStream().stream(); }

// Framework-owned high-priority side stream + the events that order it against the
// compute stream.
//  * fork()/join(): side waits for compute / compute waits for side (eager overlap, and
//    between the graph launches of a segmented captured step).
//  * record(i)/wait(i) on numbered events: under capture the event-record / event-wait
//    node is inserted explicitly into the capture graph (cross-graph ordering).
// Note (measured, profiles/overlap_r2.md): one step graph with a parallel side branch is
// executed by the HIP runtime node by node across internal streams (2.50 vs 2.13 ms per
// ResNet-18 step); and a comm graph launched after a whole compute graph starts late,
// because launching a ~200-node graph costs the host about as long as the GPU needs to
// run it.  Hence the segmented capture in utils/graph.py.
class SideStream {
 public:
  SideStream(int device, bool high_priority) : device_(device) {
    NDP_HIP_CHECK(hipSetDevice(device));
    int lo = 0, hi = 0;
    NDP_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // high priority: reducer / collective work issued mid-backward is dispatched ahead of
    // the compute stream's queued workgroups, which shortens the post-backward tail
    NDP_HIP_CHECK(hipStreamCreateWithPriority(&side_, hipStreamNonBlocking, high_priority ? hi : lo));
    ring_.resize(kRing);
    for (auto& e : ring_) NDP_HIP_CHECK(hipEventCreateWithFlags(&e, event_flags()));
  }
  ~SideStream() {
    for (auto& e : ring_) (void)hipEventDestroy(e);
    for (auto& e : named_) (void)hipEventDestroy(e);
    if (side_) (void)hipStreamDestroy(side_);
  }
  int64_t handle() const { return reinterpret_cast<int64_t>(side_); }
  int device() const { return device_; }

  // side waits for everything enqueued so far on `from` (0 = current stream)
  void fork(int64_t from) {
    hipEvent_t e = next();
    NDP_HIP_CHECK(hipEventRecord(e, pick(from)));
    NDP_HIP_CHECK(hipStreamWaitEvent(side_, e, 0));
  }
  // `into` (0 = current stream) waits for everything enqueued so far on the side stream
  void join(int64_t into) {
    hipEvent_t e = next();
    NDP_HIP_CHECK(hipEventRecord(e, side_));
    NDP_HIP_CHECK(hipStreamWaitEvent(pick(into), e, 0));
  }
  // numbered events (grown on demand) for cross-graph ordering.  Under capture the
  // event-record / event-wait node is inserted explicitly: read the stream's capture graph
  // and dependency set (hipStreamGetCaptureInfo_v2), add the node after those
  // dependencies, and make it the stream's only dependency
  // (hipStreamUpdateCaptureDependencies).  (hipEventRecordWithFlags(..External) is
  // rejected by the HIP 7.0 runtime PyTorch ships.)
  void record(int i, int64_t stream) {
    hipStream_t s = pick(stream);
    hipEvent_t e = named(i);
    if (capturing(s)) {
      insert_node(s, e, /*record=*/true);
    } else {
      NDP_HIP_CHECK(hipEventRecord(e, s));
    }
  }
  void wait(int i, int64_t stream) {
    hipStream_t s = pick(stream);
    hipEvent_t e = named(i);
    if (capturing(s)) {
      insert_node(s, e, /*record=*/false);
    } else {
      NDP_HIP_CHECK(hipStreamWaitEvent(s, e, 0));
    }
  }

 private:
  static constexpr int kRing = 64;
  static unsigned event_flags() {
    const char* v = std::getenv("NDP_EVENT_FLAGS");
    return v ? (unsigned)std::atoi(v) : hipEventDisableTiming;
  }
  static void insert_node(hipStream_t s, hipEvent_t e, bool record) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t graph = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    NDP_HIP_CHECK(hipStreamGetCaptureInfo_v2(s, &st, &id, &graph, &deps, &ndeps));
    TORCH_CHECK(st == hipStreamCaptureStatusActive && graph != nullptr, "SideStream: stream is not capturing");
    std::vector<hipGraphNode_t> d(deps, deps + ndeps);  // copy: the update below invalidates `deps`
    hipGraphNode_t node = nullptr;
    if (record) NDP_HIP_CHECK(hipGraphAddEventRecordNode(&node, graph, d.data(), d.size(), e));
    else NDP_HIP_CHECK(hipGraphAddEventWaitNode(&node, graph, d.data(), d.size(), e));
    NDP_HIP_CHECK(hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies));
  }
  hipStream_t pick(int64_t s) const { return s == 0 ? cur() : reinterpret_cast<hipStream_t>(s); }
  hipEvent_t next() {
    hipEvent_t e = ring_[next_];
    next_ = (next_ + 1) % kRing;
    return e;
  }
  hipEvent_t named(int i) {
    TORCH_CHECK(i >= 0 && i < 4096, "SideStream: event index out of range");
    while ((int)named_.size() <= i) {
      hipEvent_t e;
      NDP_HIP_CHECK(hipEventCreateWithFlags(&e, event_flags()));
      named_.push_back(e);
    }
    return named_[i];
  }
  int device_;
  hipStream_t side_ = nullptr;
  std::vector<hipEvent_t> ring_, named_;
  int next_ = 0;
};

// nodes captured so far on `stream` (0 = current); -1 if the stream is not capturing
int64_t capture_node_count(int64_t stream) {
  hipStream_t s = stream == 0 ? cur() : reinterpret_cast<hipStream_t>(stream);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  NDP_HIP_CHECK(hipStreamGetCaptureInfo_v2(s, &st, &id, &graph, &deps, &ndeps));
  if (st != hipStreamCaptureStatusActive || graph == nullptr) return -1;
  size_t n = 0;
  NDP_HIP_CHECK(hipGraphGetNodes(graph, nullptr, &n));
  return (int64_t)n;
}

}  // namespace

void register_comm(py::module& m) {
  m.def("capture_node_count", &capture_node_count, py::arg("stream") = 0);
  m.def("rccl_unique_id", &unique_id, "ncclGetUniqueId (128 bytes)");
  m.def("rccl_version", &rccl_version);
  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init<const std::string&, int, int, int>(), py::arg("uid"), py::arg("nranks"), py::arg("rank"),
           py::arg("device"))
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("device", &RcclComm::device)
      .def("all_reduce", &RcclComm::all_reduce, py::arg("t"), py::arg("op") = "sum", py::arg("stream") = 0)
      .def("all_reduce_many", &RcclComm::all_reduce_many, py::arg("ts"), py::arg("op") = "sum",
           py::arg("stream") = 0)
      .def("broadcast", &RcclComm::broadcast, py::arg("t"), py::arg("root") = 0, py::arg("stream") = 0)
      .def("all_gather", &RcclComm::all_gather, py::arg("out"), py::arg("inp"), py::arg("stream") = 0)
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::arg("out"), py::arg("inp"), py::arg("op") = "sum",
           py::arg("stream") = 0)
      .def("check", &RcclComm::check)
      .def("abort", &RcclComm::abort)
      .def("destroy", &RcclComm::destroy)
      .def_property_readonly("alive", &RcclComm::alive);
  py::class_<SideStream, std::shared_ptr<SideStream>>(m, "SideStream")
      .def(py::init<int, bool>(), py::arg("device"), py::arg("high_priority") = true)
      .def_property_readonly("handle", &SideStream::handle)
      .def_property_readonly("device", &SideStream::device)
      .def("fork", &SideStream::fork, py::arg("from_stream") = 0)
      .def("join", &SideStream::join, py::arg("into_stream") = 0)
      .def("record", &SideStream::record, py::arg("i"), py::arg("stream") = 0)
      .def("wait", &SideStream::wait, py::arg("i"), py::arg("stream") = 0);
}
