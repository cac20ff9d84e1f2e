// Native RCCL data plane for the swarm exchange rounds.
//
// One swarm round moves, per peer pair, one contiguous segment buffer plus its CRC trailer.
// Through torch.distributed that is 4 P2POps per peer (Python object, argument checks,
// group-rank translation and a Work handle each) plus a coalescing manager and a wait per
// handle: ~0.3 ms of host time per round at 7 peers, on a host path that bounds the
// per-GPU segment rate once peers share the CDN work.  Here a round is ONE call: a
// ncclGroupStart / ncclSend* / ncclRecv* / ncclGroupEnd sequence enqueued directly on the
// caller's stream (the swarm node's stream), so the transfers are stream-ordered after the
// CDN DMA / ingest CRC that produce forwarded data and before the verify CRC that consumes
// received data, with no extra streams or cross-stream events.
//
// The communicator is our own (ncclCommInitRank with an id broadcast over the control
// plane), created once per node on the ranks' devices; it links the same librccl that
// PyTorch loads (rpath to torch/lib), so the process holds one RCCL runtime.
#include <hip/hip_runtime_api.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

void nccl_ok(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

class RcclComm {
 public:
  RcclComm(const py::bytes& id_bytes, int world, int rank, int device) : world_(world), rank_(rank), device_(device) {
    const std::string id = id_bytes;
    if (id.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("RcclComm: unique id must be 128 bytes");
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("RcclComm: bad rank / world size");
    ncclUniqueId uid;
    std::memcpy(&uid, id.data(), sizeof(uid));
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // collective: blocks until every rank has joined
      if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("RcclComm: hipSetDevice failed");
      r = ncclCommInitRank(&comm_, world, uid, rank);
    }
    nccl_ok(r, "ncclCommInitRank");
  }

  // Not closed explicitly (interpreter exit): abort instead of destroy, which neither waits
  // for peers nor needs the GIL released.
  ~RcclComm() {
    if (comm_ != nullptr) ncclCommAbort(comm_);
  }

  // Post one round: every send, then every receive, inside one group on `stream`.  Per
  // (src, dst) pair the i-th send matches the i-th receive (two-sided, ordered).  The
  // buffers must stay valid until the stream reaches the transfers: the caller passes
  // views of its HBM arena or tensors allocated on the same stream (stream-ordered reuse).
  void exchange(py::array_t<int64_t, py::array::c_style | py::array::forcecast> send_ptr,
                py::array_t<int64_t, py::array::c_style | py::array::forcecast> send_bytes,
                py::array_t<int64_t, py::array::c_style | py::array::forcecast> send_peer,
                py::array_t<int64_t, py::array::c_style | py::array::forcecast> recv_ptr,
                py::array_t<int64_t, py::array::c_style | py::array::forcecast> recv_bytes,
                py::array_t<int64_t, py::array::c_style | py::array::forcecast> recv_peer, int64_t stream) {
    if (comm_ == nullptr) throw std::runtime_error("RcclComm: communicator is closed");
    const int64_t ns = send_ptr.size(), nr = recv_ptr.size();
    if (send_bytes.size() != ns || send_peer.size() != ns || recv_bytes.size() != nr || recv_peer.size() != nr)
      throw std::invalid_argument("RcclComm.exchange: argument sizes differ");
    const int64_t *sp = send_ptr.data(), *sb = send_bytes.data(), *sd = send_peer.data();
    const int64_t *rp = recv_ptr.data(), *rb = recv_bytes.data(), *rs = recv_peer.data();
    for (int64_t i = 0; i < ns; ++i)
      if (sd[i] < 0 || sd[i] >= world_ || sb[i] < 0) throw std::invalid_argument("RcclComm.exchange: bad send");
    for (int64_t i = 0; i < nr; ++i)
      if (rs[i] < 0 || rs[i] >= world_ || rb[i] < 0) throw std::invalid_argument("RcclComm.exchange: bad recv");
    if (ns == 0 && nr == 0) return;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    ncclResult_t r = ncclSuccess;
    {
      py::gil_scoped_release nogil;
      r = ncclGroupStart();
      for (int64_t i = 0; r == ncclSuccess && i < ns; ++i)
        if (sb[i] > 0)
          r = ncclSend(reinterpret_cast<const void*>(sp[i]), static_cast<size_t>(sb[i]), ncclUint8,
                       static_cast<int>(sd[i]), comm_, st);
      for (int64_t i = 0; r == ncclSuccess && i < nr; ++i)
        if (rb[i] > 0)
          r = ncclRecv(reinterpret_cast<void*>(rp[i]), static_cast<size_t>(rb[i]), ncclUint8,
                       static_cast<int>(rs[i]), comm_, st);
      const ncclResult_t e = ncclGroupEnd();  // always closes the group, even after an error
      if (r == ncclSuccess) r = e;
    }
    nccl_ok(r, "send/recv group");
    ++rounds_;
  }

  // Asynchronous error state of the communicator (a peer failure surfaces here).
  std::string async_error() {
    if (comm_ == nullptr) return "";
    ncclResult_t a = ncclSuccess;
    nccl_ok(ncclCommGetAsyncError(comm_, &a), "ncclCommGetAsyncError");
    return a == ncclSuccess ? "" : ncclGetErrorString(a);
  }

  void close() {
    if (comm_ == nullptr) return;
    ncclComm_t c = comm_;
    comm_ = nullptr;
    py::gil_scoped_release nogil;
    ncclCommDestroy(c);  // waits for this rank's outstanding transfers
  }

  // Tear down without waiting for peers (error paths, interpreter exit).
  void abort() {
    if (comm_ == nullptr) return;
    ncclComm_t c = comm_;
    comm_ = nullptr;
    ncclCommAbort(c);
  }

  // What RCCL itself reports for this communicator (the topology record of an N > 1 run
  // proves the group RCCL built, not the one the caller asked for): its rank count, this
  // rank's index in it, and the HIP device it runs on.
  int comm_count() const {
    int n = 0;
    nccl_ok(ncclCommCount(live(), &n), "ncclCommCount");
    return n;
  }
  int comm_user_rank() const {
    int r = -1;
    nccl_ok(ncclCommUserRank(live(), &r), "ncclCommUserRank");
    return r;
  }
  int comm_device() const {
    int d = -1;
    nccl_ok(ncclCommCuDevice(live(), &d), "ncclCommCuDevice");
    return d;
  }

  bool closed() const { return comm_ == nullptr; }
  int world() const { return world_; }
  int rank() const { return rank_; }
  int device() const { return device_; }
  int64_t rounds() const { return rounds_; }

 private:
  ncclComm_t live() const {
    if (comm_ == nullptr) throw std::runtime_error("RcclComm: communicator is closed");
    return comm_;
  }
  ncclComm_t comm_ = nullptr;
  int world_, rank_, device_;
  int64_t rounds_ = 0;
};

py::bytes unique_id() {
  ncclUniqueId uid;
  nccl_ok(ncclGetUniqueId(&uid), "ncclGetUniqueId");
  return py::bytes(reinterpret_cast<const char*>(&uid), sizeof(uid));
}

std::string version() {
  int v = 0;
  nccl_ok(ncclGetVersion(&v), "ncclGetVersion");
  return std::to_string(v);
}

// PCI address ("dddd:bb:dd.f") of a HIP device: the identity two ranks compare to prove they
// drive different GPUs (a device index is only meaningful inside one process's visible set).
std::string pci_bus_id(int device) {
  char buf[64] = {0};
  if (hipDeviceGetPCIBusId(buf, sizeof(buf), device) != hipSuccess)
    throw std::runtime_error("hipDeviceGetPCIBusId failed for device " + std::to_string(device));
  return std::string(buf);
}

// HIP's view of the link between two devices of this process (HSA_AMD_LINK_INFO_TYPE_*:
// 2 = PCIe, 4 = xGMI) and its hop count: the second, RCCL-independent proof of the wire an
// N > 1 record ran on (parallel/wire.py).
py::tuple link_type(int dev_a, int dev_b) {
  uint32_t type = 0, hops = 0;
  const hipError_t e = hipExtGetLinkTypeAndHopCount(dev_a, dev_b, &type, &hops);
  if (e != hipSuccess)
    throw std::runtime_error(std::string("hipExtGetLinkTypeAndHopCount: ") + hipGetErrorString(e));
  return py::make_tuple(type, hops);
}

}  // namespace

void register_rccl(py::module& m) {
  m.def("rccl_unique_id", &unique_id, "ncclGetUniqueId (rank 0 of a new communicator)");
  m.def("rccl_version", &version);
  m.def("pci_bus_id", &pci_bus_id, py::arg("device"));
  m.def("link_type", &link_type, py::arg("dev_a"), py::arg("dev_b"));
  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init<const py::bytes&, int, int, int>(), py::arg("unique_id"), py::arg("world"), py::arg("rank"),
           py::arg("device"))
      .def("exchange", &RcclComm::exchange, py::arg("send_ptr"), py::arg("send_bytes"), py::arg("send_peer"),
           py::arg("recv_ptr"), py::arg("recv_bytes"), py::arg("recv_peer"), py::arg("stream"))
      .def("async_error", &RcclComm::async_error)
      .def("close", &RcclComm::close)
      .def("abort", &RcclComm::abort)
      .def_property_readonly("closed", &RcclComm::closed)
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("device", &RcclComm::device)
      .def_property_readonly("rounds", &RcclComm::rounds)
      .def("comm_count", &RcclComm::comm_count)
      .def("comm_user_rank", &RcclComm::comm_user_rank)
      .def("comm_device", &RcclComm::comm_device);
}
