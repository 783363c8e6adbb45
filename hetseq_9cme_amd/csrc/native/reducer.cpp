// Native gradient reducer: the bucket state machine behind parallel/reducer.py.
//
// Replaces the C++ reducer of torch.nn.parallel.DistributedDataParallel that the reference
// wraps its model in (hetseq/controller.py:75-90).  Design for this
// framework's flat layout (parallel/flat_params.py):
//
//  * every trainable parameter's gradient lives in ONE flat buffer; a bucket is a
//    contiguous [start, end) slice of it, reduced IN PLACE (no pack / unpack copies);
//  * a C++ post-accumulate-grad hook per parameter (no Python on the per-parameter path)
//    makes the parameter's .grad its flat slot (a no-op when a fused backward kernel
//    already wrote the gradient there), counts the bucket down and launches every bucket
//    that is complete, strictly in index order -- the identical collective sequence on
//    every rank, whatever order the gradients arrive in;
//  * an autograd-engine final callback flushes buckets holding parameters this rank did
//    not use (their slots are zero-filled) and makes the compute stream wait for the
//    collectives: no host blocking on the GPU path;
//  * transports: any c10d ProcessGroup (RCCL -- "nccl" on ROCm -- between MI355X GPUs,
//    gloo for CPU runs and tests), or the hand-written intra-node xGMI two-shot kernel
//    (csrc/kernels/xgmi_allreduce.hip) on a high-priority comm stream that waits for the
//    producing stream(s) through HIP events;
//  * single-process runs keep the hooks (they record the used flags; nothing is reduced):
//    gradient version counters cannot tell, since every slot is a view of the one flat
//    buffer and views share their base's version counter.
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/function_hook.h>
#include <torch/csrc/autograd/variable.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/distributed/c10d/Work.hpp>
#include <torch/extension.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <vector>

#include "hx_launch.h"

namespace hx {
namespace {

using torch::Tensor;

// Side stream of the running backward (``--overlap-wgrad``: ops/fused.py side_begin /
// side_join publish it), so a bucket's collective is ordered after the weight-gradient
// GEMMs queued there.
std::atomic<hipStream_t> g_side_stream{nullptr};

inline void hip_ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "reducer: ", what, " failed: ", hipGetErrorString(e));
}

class Reducer : public std::enable_shared_from_this<Reducer> {
 public:
  Reducer(Tensor grad_flat, std::vector<Tensor> params, std::vector<int64_t> offsets, std::vector<int64_t> bounds,
          std::vector<int64_t> bucket_of, c10::intrusive_ptr<c10d::ProcessGroup> pg, int64_t world, bool force)
      : grad_flat_(std::move(grad_flat)), params_(std::move(params)), pg_(std::move(pg)), world_(world),
        force_(force) {
    const size_t P = params_.size();
    TORCH_CHECK(offsets.size() == P && bucket_of.size() == P, "reducer: one offset / bucket per parameter");
    TORCH_CHECK(bounds.size() >= 2, "reducer: at least one bucket");
    nb_ = (int)bounds.size() - 1;
    for (int b = 0; b < nb_; ++b) {
      TORCH_CHECK(bounds[b] <= bounds[b + 1] && bounds[b + 1] <= grad_flat_.numel(), "reducer: bad bucket bounds");
    }
    bounds_ = std::move(bounds);
    bucket_of_.assign(bucket_of.begin(), bucket_of.end());
    nparams_.assign(nb_, 0);
    slots_.reserve(P);
    for (size_t i = 0; i < P; ++i) {
      TORCH_CHECK(bucket_of_[i] >= 0 && bucket_of_[i] < nb_, "reducer: bucket index out of range");
      ++nparams_[bucket_of_[i]];
      const Tensor& p = params_[i];
      TORCH_CHECK(offsets[i] >= 0 && offsets[i] + p.numel() <= grad_flat_.numel(), "reducer: slot out of range");
      slots_.push_back(grad_flat_.narrow(0, offsets[i], p.numel()).view(p.sizes()));
    }
    enabled_ = (world_ > 1 || force_) && pg_;
    used_.assign(P, 0);
    reset_iteration();
    if (grad_flat_.is_cuda()) {
      c10::hip::HIPGuardMasqueradingAsCUDA guard(grad_flat_.device());
      hip_ok(hipEventCreateWithFlags(&ev_, hipEventDisableTiming), "hipEventCreate");
    }
  }

  ~Reducer() {
    remove_hooks();
    if (ev_) (void)hipEventDestroy(ev_);
  }

  // ---------------------------------------------------------------- hooks
  struct Hook : torch::autograd::PostAccumulateGradHook {
    Hook(std::weak_ptr<Reducer> r, int i) : r_(std::move(r)), i_(i) {}
    void operator()(const torch::autograd::Variable& p) override {
      if (auto r = r_.lock()) r->grad_ready(i_, p);
    }
    std::weak_ptr<Reducer> r_;
    int i_;
  };

  void install_hooks() {
    if (hooks_installed_) return;
    std::weak_ptr<Reducer> self = weak_from_this();
    for (size_t i = 0; i < params_.size(); ++i) {
      TORCH_CHECK(params_[i].is_leaf() && params_[i].requires_grad(), "reducer: parameters must be leaves");
      torch::autograd::impl::set_post_acc_grad_hooks(params_[i], std::make_unique<Hook>(self, (int)i));
    }
    hooks_installed_ = true;
  }

  void remove_hooks() {
    if (!hooks_installed_) return;
    for (auto& p : params_) torch::autograd::impl::set_post_acc_grad_hooks(p, nullptr);
    hooks_installed_ = false;
  }

  void grad_ready(int i, const Tensor& p) {
    std::lock_guard<std::mutex> lk(mu_);
    if (used_[i]) return;   // accumulated twice in one backward (reentrant use)
    used_[i] = 1;
    adopt(i, p);
    if (!callback_queued_) {
      callback_queued_ = true;
      std::weak_ptr<Reducer> self = weak_from_this();
      torch::autograd::Engine::get_default_engine().queue_callback([self]() {
        if (auto r = self.lock()) {
          std::lock_guard<std::mutex> lk2(r->mu_);
          r->finalize_locked();
        }
      });
    }
    if (!(enabled_ && sync_)) return;
    --pending_[bucket_of_[i]];
    launch_ready(false);
  }

  // ---------------------------------------------------------------- per-iteration API
  // Before each micro-batch's forward: returns the previous micro-batch's used flags.
  std::vector<bool> prepare() {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<bool> prev(used_.begin(), used_.end());
    reset_iteration();
    return prev;
  }

  // After each micro-batch's backward.  When no hook fired (the loss reached no parameter),
  // finalize here so this rank still joins every bucket collective.
  void after_backward() {
    std::lock_guard<std::mutex> lk(mu_);
    if (!callback_queued_) {
      callback_queued_ = true;
      finalize_locked();
    }
  }

  void set_sync(bool s) {
    std::lock_guard<std::mutex> lk(mu_);
    sync_ = s;
  }
  bool sync() const { return sync_; }

  std::vector<bool> used() {
    std::lock_guard<std::mutex> lk(mu_);
    return std::vector<bool>(used_.begin(), used_.end());
  }

  // Reduce the whole gradient buffer now (a rank that ran no backward this update).
  void all_reduce_now() {
    std::lock_guard<std::mutex> lk(mu_);
    if (!enabled_) return;
    if (xar_) {
      c10::hip::HIPGuardMasqueradingAsCUDA guard(grad_flat_.device());
      const hipStream_t cur = c10::hip::getCurrentHIPStream(grad_flat_.get_device()).stream();
      hip_ok(hipEventRecord(ev_, cur), "hipEventRecord");
      hip_ok(hipStreamWaitEvent(comm_, ev_, 0), "hipStreamWaitEvent");
      TORCH_CHECK(hx_xar_allreduce(xar_, grad_flat_.data_ptr<float>(), grad_flat_.numel(), comm_) == 0,
                  hx_xar_last_error());
      hip_ok(hipEventRecord(ev_, comm_), "hipEventRecord");
      hip_ok(hipStreamWaitEvent(cur, ev_, 0), "hipStreamWaitEvent");
    } else {
      std::vector<Tensor> ts{grad_flat_};
      pg_->allreduce(ts)->wait();
    }
  }

  void use_xgmi(int64_t ctx, int64_t comm_stream) {
    std::lock_guard<std::mutex> lk(mu_);
    TORCH_CHECK(grad_flat_.is_cuda() && grad_flat_.scalar_type() == torch::kFloat32,
                "xGMI transport: fp32 GPU gradients only");
    xar_ = reinterpret_cast<void*>(static_cast<uintptr_t>(ctx));
    comm_ = reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(comm_stream));
  }
  void drop_xgmi() {
    std::lock_guard<std::mutex> lk(mu_);
    xar_ = nullptr;
    comm_ = nullptr;
  }

  // --use-bmuf: hooks keep adopting slots / recording used flags, nothing is reduced
  void set_enabled(bool on) {
    std::lock_guard<std::mutex> lk(mu_);
    enabled_ = on && (world_ > 1 || force_) && pg_;
  }

  // --comm-cus: CUs the compute plans leave to the collectives while buckets are in flight
  void set_comm_cus(int64_t n) {
    std::lock_guard<std::mutex> lk(mu_);
    comm_cus_ = (int)std::max<int64_t>(0, n);
  }

  int num_buckets() const { return nb_; }
  int launched() const { return launched_; }
  bool enabled() const { return enabled_; }

 private:
  void reset_iteration() {
    if (reserving_) {   // a backward that raised before finalize_locked(): give the CUs back
      hx_set_reserved_cus(0);
      reserving_ = false;
    }
    pending_ = nparams_;
    launched_ = 0;
    works_.clear();
    callback_queued_ = false;
    std::fill(used_.begin(), used_.end(), 0);
  }

  // param i's .grad becomes its flat slot: copy a gradient produced elsewhere in,
  // zero-fill when the parameter got none this micro-batch
  void adopt(int i, const Tensor& p) {
    Tensor& g = p.mutable_grad();
    const Tensor& slot = slots_[i];
    if (!g.defined()) {
      slot.zero_();
      g = slot;
    } else if (g.data_ptr() != slot.data_ptr()) {
      slot.copy_(g);
      g = slot;
    }
  }

  void launch_ready(bool force) {
    while (launched_ < nb_ && (force || pending_[launched_] == 0)) {
      launch_bucket(launched_);
      ++launched_;
    }
  }

  void launch_bucket(int b) {
    const int64_t s = bounds_[b], n = bounds_[b + 1] - bounds_[b];
    if (n == 0) return;
    if (comm_cus_ > 0 && grad_flat_.is_cuda() && !reserving_) {
      // from the first collective of this backward to its end, the GEMM / weight-gradient plans
      // leave comm_cus_ CUs to the all-reduce (cu_reserve.hip); finalize_locked() gives them back
      hx_set_reserved_cus(comm_cus_);
      reserving_ = true;
    }
    Tensor view = grad_flat_.narrow(0, s, n);
    if (!grad_flat_.is_cuda()) {   // CPU (gloo): no streams
      std::vector<Tensor> ts{view};
      works_.push_back(pg_->allreduce(ts));
      return;
    }
    c10::hip::HIPGuardMasqueradingAsCUDA guard(grad_flat_.device());
    const int dev = grad_flat_.get_device();
    const hipStream_t cur = c10::hip::getCurrentHIPStream(dev).stream();
    const hipStream_t side = g_side_stream.load();
    if (xar_) {
      hip_ok(hipEventRecord(ev_, cur), "hipEventRecord");
      hip_ok(hipStreamWaitEvent(comm_, ev_, 0), "hipStreamWaitEvent");
      if (side) {
        hip_ok(hipEventRecord(ev_, side), "hipEventRecord");
        hip_ok(hipStreamWaitEvent(comm_, ev_, 0), "hipStreamWaitEvent");
      }
      TORCH_CHECK(hx_xar_allreduce(xar_, view.data_ptr<float>(), n, comm_) == 0, hx_xar_last_error());
      return;
    }
    std::vector<Tensor> ts{view};
    if (side) {
      // the bucket's weight gradients may come from the side stream: launch the collective
      // from it, after everything the compute stream queued so far
      hip_ok(hipEventRecord(ev_, cur), "hipEventRecord");
      hip_ok(hipStreamWaitEvent(side, ev_, 0), "hipStreamWaitEvent");
      c10::hip::HIPStreamGuardMasqueradingAsCUDA sg(
          c10::hip::getStreamFromExternalMasqueradingAsCUDA(side, static_cast<c10::DeviceIndex>(dev)));
      works_.push_back(pg_->allreduce(ts));
    } else {
      works_.push_back(pg_->allreduce(ts));
    }
  }

  void finalize_locked() {
    for (size_t i = 0; i < params_.size(); ++i)
      if (!used_[i]) adopt((int)i, params_[i]);   // unused this micro-batch: keep / zero its slot
    if (enabled_ && sync_) {
      launch_ready(true);   // buckets with unused parameters: their slices hold zeros
      if (xar_) {
        c10::hip::HIPGuardMasqueradingAsCUDA guard(grad_flat_.device());
        const hipStream_t cur = c10::hip::getCurrentHIPStream(grad_flat_.get_device()).stream();
        hip_ok(hipEventRecord(ev_, comm_), "hipEventRecord");
        hip_ok(hipStreamWaitEvent(cur, ev_, 0), "hipStreamWaitEvent");
      }
      for (auto& w : works_) w->wait();   // RCCL: the current stream waits, the host does not
    }
    works_.clear();
    if (reserving_) {
      hx_set_reserved_cus(0);
      reserving_ = false;
    }
  }

  Tensor grad_flat_;
  std::vector<Tensor> params_, slots_;
  std::vector<int64_t> bounds_;
  std::vector<int> bucket_of_, nparams_, pending_;
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  int64_t world_;
  bool force_ = false;   // reduce even in a one-rank group (tests drive the RCCL stream path on one GPU)
  int comm_cus_ = 0;
  bool reserving_ = false;
  bool hooks_installed_ = false;
  bool enabled_ = false;
  bool sync_ = true;
  bool callback_queued_ = false;
  int nb_ = 0, launched_ = 0;
  std::vector<uint8_t> used_;
  std::vector<c10::intrusive_ptr<c10d::Work>> works_;
  void* xar_ = nullptr;
  hipStream_t comm_ = nullptr;
  hipEvent_t ev_ = nullptr;
  std::mutex mu_;
};

std::shared_ptr<Reducer> make_reducer(Tensor grad_flat, std::vector<Tensor> params, std::vector<int64_t> offsets,
                                      std::vector<int64_t> bounds, std::vector<int64_t> bucket_of,
                                      py::object process_group, int64_t world, bool force) {
  c10::intrusive_ptr<c10d::ProcessGroup> pg;
  if (!process_group.is_none()) pg = process_group.cast<c10::intrusive_ptr<c10d::ProcessGroup>>();
  auto r = std::make_shared<Reducer>(std::move(grad_flat), std::move(params), std::move(offsets), std::move(bounds),
                                     std::move(bucket_of), std::move(pg), world, force);
  r->install_hooks();
  return r;
}

void set_side_stream(int64_t handle) {
  g_side_stream.store(reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(handle)));
}

}  // namespace

void register_reducer(py::module& m) {
  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init(&make_reducer), py::arg("grad_flat"), py::arg("params"), py::arg("offsets"), py::arg("bounds"),
           py::arg("bucket_of"), py::arg("process_group"), py::arg("world"), py::arg("force") = false)
      // the GIL is released wherever a call may wait for a collective or run torch ops whose
      // tensors' Python owners the collectives' worker threads may need to release
      .def("prepare", &Reducer::prepare, py::call_guard<py::gil_scoped_release>())
      .def("after_backward", &Reducer::after_backward, py::call_guard<py::gil_scoped_release>())
      .def("set_sync", &Reducer::set_sync)
      .def("sync", &Reducer::sync)
      .def("used", &Reducer::used)
      .def("all_reduce_now", &Reducer::all_reduce_now, py::call_guard<py::gil_scoped_release>())
      .def("use_xgmi", &Reducer::use_xgmi)
      .def("drop_xgmi", &Reducer::drop_xgmi)
      .def("remove_hooks", &Reducer::remove_hooks)
      .def("set_enabled", &Reducer::set_enabled)
      .def("set_comm_cus", &Reducer::set_comm_cus)
      .def("num_buckets", &Reducer::num_buckets)
      .def("launched", &Reducer::launched)
      .def("enabled", &Reducer::enabled);
  m.def("reducer_set_side_stream", &set_side_stream);
}

}  // namespace hx
