// Python bindings of the peer-mapped all-reduce (csrc/kernels/comm.hip): buffer allocation, IPC
// handle export / import and the launch.  parallel/p2p.py drives it (handle exchange over the
// process group, epoch counting, status checks).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <cstring>
#include <string>
#include <vector>

#include "avenir_kernels.h"

namespace {

using DevGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

void hip_ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "p2p: ", what, " failed: ", hipGetErrorString(e));
}

constexpr size_t kFlagWords = (size_t)avk::P2P_MAX_RANKS * avk::P2P_MAX_BLOCKS;

class P2PComm {
 public:
  P2PComm(int64_t device, int64_t cap_bytes, bool uncached_data) : device_((int)device) {
    TORCH_CHECK(cap_bytes > 0 && cap_bytes <= (int64_t(1) << 31), "p2p: cap_bytes out of range");
    cap_ = (cap_bytes + 255) / 256 * 256;
    DevGuard g(c10::Device(c10::DeviceType::CUDA, device_));
    if (uncached_data)
      hip_ok(hipExtMallocWithFlags(&data_, 4 * (size_t)cap_, hipDeviceMallocUncached), "data alloc");
    else
      hip_ok(hipMalloc(&data_, 4 * (size_t)cap_), "data alloc");
    // flag words + the status word, uncached so polls read HBM
    void* f = nullptr;
    hip_ok(hipExtMallocWithFlags(&f, kFlagWords * sizeof(unsigned) + 256, hipDeviceMallocUncached), "flag alloc");
    flags_ = static_cast<unsigned*>(f);
    status_ = reinterpret_cast<int*>(flags_ + kFlagWords);
    hip_ok(hipMemset(flags_, 0, kFlagWords * sizeof(unsigned) + 256), "flag memset");
    // the host-visible status word: pinned, coherent and mapped, so the host reads a kernel's
    // verdict once the kernel has finished without synchronising the device
    void* hs = nullptr;
    hip_ok(hipHostMalloc(&hs, 256, hipHostMallocMapped | hipHostMallocCoherent), "host status alloc");
    host_status_ = static_cast<volatile int*>(hs);
    *host_status_ = 0;
    void* hsd = nullptr;
    hip_ok(hipHostGetDevicePointer(&hsd, hs, 0), "host status device pointer");
    host_status_dev_ = static_cast<int*>(hsd);
    hip_ok(hipEventCreateWithFlags(&last_, hipEventDisableTiming), "event create");
    hip_ok(hipMemset(data_, 0, 4 * (size_t)cap_), "data memset");
    hip_ok(hipDeviceSynchronize(), "sync");
    int khz = 0;
    hip_ok(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_), "wall clock rate");
    clock_khz_ = khz > 0 ? khz : 100000;
    set_timeout(10.0);
    std::memset(&view_, 0, sizeof(view_));
  }

  // no implicit release: at interpreter exit the HIP runtime may already be gone (the OS reclaims the
  // mappings); parallel/p2p.py closes peers, barriers and releases explicitly
  ~P2PComm() = default;

  int64_t cap_bytes() const { return cap_; }

  // 2 x HIP_IPC_HANDLE_SIZE bytes: the data region's handle, then the flag region's
  py::bytes handles() const {
    hipIpcMemHandle_t hd, hf;
    hip_ok(hipIpcGetMemHandle(&hd, data_), "ipc handle (data)");
    hip_ok(hipIpcGetMemHandle(&hf, flags_), "ipc handle (flags)");
    std::string s(reinterpret_cast<const char*>(&hd), sizeof(hd));
    s.append(reinterpret_cast<const char*>(&hf), sizeof(hf));
    return py::bytes(s);
  }

  void open(const std::vector<std::string>& all, int64_t rank, int64_t world) {
    TORCH_CHECK(!open_, "p2p: peers already opened");
    TORCH_CHECK(world >= 1 && world <= avk::P2P_MAX_RANKS, "p2p: world must be in [1, ", avk::P2P_MAX_RANKS, "]");
    TORCH_CHECK(rank >= 0 && rank < world && (int64_t)all.size() == world, "p2p: bad rank / handle list");
    DevGuard g(c10::Device(c10::DeviceType::CUDA, device_));
    view_.rank = (int)rank;
    view_.world = (int)world;
    view_.cap_bytes = cap_;
    view_.status = status_;
    view_.host_status = host_status_dev_;
    for (int64_t k = 0; k < world; ++k) {
      if (k == rank) {
        view_.data[k] = data_;
        view_.flags[k] = flags_;
        continue;
      }
      TORCH_CHECK(all[k].size() == 2 * sizeof(hipIpcMemHandle_t), "p2p: handle of rank ", k, " has bad size");
      hipIpcMemHandle_t hd, hf;
      std::memcpy(&hd, all[k].data(), sizeof(hd));
      std::memcpy(&hf, all[k].data() + sizeof(hd), sizeof(hf));
      void* pd = nullptr;
      void* pf = nullptr;
      hip_ok(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess), "ipc open (data)");
      opened_.push_back(pd);
      hip_ok(hipIpcOpenMemHandle(&pf, hf, hipIpcMemLazyEnablePeerAccess), "ipc open (flags)");
      opened_.push_back(pf);
      view_.data[k] = pd;
      view_.flags[k] = static_cast<unsigned*>(pf);
    }
    open_ = true;
  }

  void set_timeout(double seconds) {
    TORCH_CHECK(seconds > 0 && seconds < 1e7, "p2p: timeout out of range");
    timeout_ticks_ = (int64_t)(seconds * clock_khz_ * 1000.0);
  }

  // in-place sum of t over all ranks; epoch >= 1, strictly increasing by 1 per call on every rank
  void all_reduce(at::Tensor& t, int64_t epoch, bool two_shot) {
    TORCH_CHECK(open_, "p2p: open() the peers first");
    TORCH_CHECK(t.is_cuda() && t.device().index() == device_, "p2p: tensor must live on the communicator's device");
    TORCH_CHECK(t.is_contiguous(), "p2p: tensor must be contiguous");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "p2p: tensor must be 16-byte aligned");
    TORCH_CHECK(epoch >= 1 && epoch <= avk::P2P_MAX_EPOCH, "p2p: epoch out of range");
    int dt;
    switch (t.scalar_type()) {
      case at::kFloat: dt = avk::P2P_F32; break;
      case at::kDouble: dt = avk::P2P_F64; break;
      case at::kInt: dt = avk::P2P_I32; break;
      case at::kLong: dt = avk::P2P_I64; break;
      default: TORCH_CHECK(false, "p2p: dtype must be float32, float64, int32 or int64");
    }
    const int64_t nbytes = t.numel() * t.element_size();
    TORCH_CHECK(nbytes <= cap_, "p2p: message of ", nbytes, " bytes exceeds the staging capacity ", cap_);
    DevGuard g(t.device());
    hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(device_).stream();
    // the staging parities are reused by epoch order, so consecutive calls must run in order: a
    // call issued on another stream than the previous one first waits for that one
    if (have_last_ && st != last_stream_) hip_ok(hipStreamWaitEvent(st, last_, 0), "stream wait");
    avk::p2p_all_reduce(t.data_ptr(), t.numel(), dt, view_, (unsigned)epoch, two_shot ? 1 : 0, timeout_ticks_, st);
    hip_ok(hipEventRecord(last_, st), "event record");
    last_stream_ = st;
    have_last_ = true;
  }

  // the host-visible status of the kernels that have FINISHED: 0 healthy, 1 a wait here timed out,
  // 2 a peer reported a failure (no device synchronisation)
  int64_t host_status() const { return host_status_ != nullptr ? *host_status_ : 0; }

  // block the host until the last call's kernel has finished
  void sync_last() const {
    if (have_last_) hip_ok(hipEventSynchronize(last_), "event sync");
  }

  // true when the last call's kernel has finished (hipEventQuery; no synchronisation)
  bool last_done() const { return !have_last_ || hipEventQuery(last_) == hipSuccess; }

  // poison this rank's flags in every peer (their next wait on us ends with status 2), then wait
  // for it: the failing rank's last act on the channel before it raises
  void poison() {
    TORCH_CHECK(open_, "p2p: open() the peers first");
    DevGuard g(c10::Device(c10::DeviceType::CUDA, device_));
    hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(device_).stream();
    if (have_last_ && st != last_stream_) hip_ok(hipStreamWaitEvent(st, last_, 0), "stream wait");
    avk::p2p_poison(view_, st);
    hip_ok(hipStreamSynchronize(st), "poison sync");
  }

  // 0 = healthy; 1 = a wait timed out; 2 = a peer failed (synchronises the device)
  int64_t status() const {
    int s = 0;
    DevGuard g(c10::Device(c10::DeviceType::CUDA, device_));
    hip_ok(hipMemcpy(&s, status_, sizeof(int), hipMemcpyDeviceToHost), "status read");
    return s;
  }

  // unmap the peers' regions (call on every rank, then barrier, then free())
  void close_peers() {
    DevGuard g(c10::Device(c10::DeviceType::CUDA, device_));
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    opened_.clear();
    open_ = false;
  }

  void release() {
    if (data_ == nullptr && flags_ == nullptr) return;
    close_peers();
    (void)hipFree(data_);
    (void)hipFree(flags_);
    if (host_status_ != nullptr) (void)hipHostFree(const_cast<int*>(host_status_));
    if (last_ != nullptr) (void)hipEventDestroy(last_);
    data_ = nullptr;
    flags_ = nullptr;
    status_ = nullptr;
    host_status_ = nullptr;
    host_status_dev_ = nullptr;
    last_ = nullptr;
    have_last_ = false;
  }

 private:
  int device_;
  int64_t cap_ = 0;
  void* data_ = nullptr;
  unsigned* flags_ = nullptr;
  int* status_ = nullptr;
  volatile int* host_status_ = nullptr;
  int* host_status_dev_ = nullptr;
  hipEvent_t last_ = nullptr;
  hipStream_t last_stream_ = nullptr;
  bool have_last_ = false;
  int clock_khz_ = 100000;
  int64_t timeout_ticks_ = 0;
  bool open_ = false;
  std::vector<void*> opened_;
  avk::P2PView view_;
};

}  // namespace

void register_comm(py::module_& m) {
  py::class_<P2PComm>(m, "P2PComm")
      .def(py::init<int64_t, int64_t, bool>(), py::arg("device"), py::arg("cap_bytes"), py::arg("uncached_data") = false)
      .def_property_readonly("cap_bytes", &P2PComm::cap_bytes)
      .def("handles", &P2PComm::handles)
      .def("open", &P2PComm::open)
      .def("set_timeout", &P2PComm::set_timeout)
      .def("all_reduce", &P2PComm::all_reduce)
      .def("status", &P2PComm::status)
      .def("host_status", &P2PComm::host_status)
      .def("last_done", &P2PComm::last_done)
      .def("sync_last", &P2PComm::sync_last, py::call_guard<py::gil_scoped_release>())
      .def("poison", &P2PComm::poison)
      .def("close_peers", &P2PComm::close_peers)
      .def("release", &P2PComm::release);
}
