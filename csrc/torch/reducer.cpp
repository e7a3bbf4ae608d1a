// DDP gradient reducer core (apex.parallel.DistributedDataParallel semantics).
//
// Behavioural spec: apex@f3a960f8 apex/parallel/distributed.py (SURVEY.md A-14,
// call stack §3.4).  MI355X-native design:
//  * gradients live as VIEWS into persistent per-bucket flat buffers
//    (param.grad aliases the bucket), so apex_C.flatten / unflatten copies and
//    the multi_tensor_scale "unflatten" pass disappear;
//  * the grad-ready hook is a C++ post-hook on each parameter's AccumulateGrad
//    node (no Python, no GIL on the backward critical path);
//  * a bucket is handed to the process group (RCCL over xGMI on MI355X; gloo on
//    CPU) the moment it is complete AND every earlier bucket has been launched,
//    so all ranks issue collectives in the same order; ProcessGroupNCCL runs
//    them on its own stream, overlapped with the rest of backward;
//  * averaging uses ncclAvg (ReduceOp::AVG) when possible -> no post-scale pass;
//  * iteration 1 records the real grad-arrival order, rank 0 broadcasts it
//    (apex sync_bucket_structure) and the buckets are rebuilt in that order;
//  * end-of-backward epilogue (engine final callback) makes the compute stream
//    wait on every bucket's collective and checks that every bucket was reduced;
//  * the process group handed in by the Python wrapper is a dedicated
//    communicator created with high-priority HIP streams (ProcessGroupNCCL
//    Options.is_high_priority_stream), so bucket all-reduces are scheduled ahead
//    of backward kernels and never queue behind user / SyncBN collectives;
//  * `force_collectives` issues the all-reduce even on a 1-rank communicator
//    (legal on RCCL): the single-GPU test box then exercises launch order, the
//    epilogue stream join and in-flight bucket consumption for real;
//  * gradients produced on a SIDE stream (ops/conv.py weight gradients overlapping
//    the data gradient) are accumulated into their bucket views on that stream and
//    announced with `mark_ready_on_stream`: the reducer records an event there,
//    and a bucket holding such gradients is launched from an internal launch stream
//    that waits on the compute stream AND those events - the compute stream itself
//    never waits for the side stream before the end-of-backward join;
//  * `prof` (apex prof=True): roctx ranges around every bucket launch and the
//    epilogue (visible in rocprofv3 --marker-trace next to the kernels);
//  * optional per-bucket timing (HIP events on the compute stream): when each
//    bucket was launched relative to the first gradient, when backward ended,
//    and when each bucket's collective was joined -> the exposed
//    post-backward communication tail that bench.py reports at N > 1.
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/utils/lambda_post_hook.h>
#include <torch/csrc/autograd/variable.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/extension.h>
#include <ATen/record_function.h>

#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <memory>
#include <mutex>
#include <string>

#include "reducer.h"
#include "norm_ops.h"

extern "C" int roctxRangePushA(const char* message);  // libroctx64 (what torch.cuda.nvtx uses)
extern "C" int roctxRangePop();

namespace amd {

namespace {

struct Bucket {
  at::ScalarType dtype;
  std::vector<int64_t> params;
  std::vector<int64_t> offsets;
  int64_t numel = 0;
  at::Tensor flat;
  at::Tensor comm;
  int pending = 0;
  bool launched = false;
  c10::intrusive_ptr<c10d::Work> work;
  std::vector<hipEvent_t> waits;  // side-stream gradient events this launch must wait on
  bool split = false;  // reduced as fp32 reduce-scatter + 16-bit all-gather (fp32 mode 3)
  at::Tensor shard;    // that reduce-scatter's fp32 output (kept until the join)
};

struct RangeGuard {  // roctx range when enabled
  bool on;
  RangeGuard(bool e, const std::string& name) : on(e) {
    if (on) roctxRangePushA(name.c_str());
  }
  ~RangeGuard() {
    if (on) roctxRangePop();
  }
};

class Reducer;
struct SideWaitPreHook : torch::autograd::FunctionPreHook {
  SideWaitPreHook(std::weak_ptr<Reducer> r, int64_t i) : red(std::move(r)), idx(i) {}
  torch::autograd::variable_list operator()(const torch::autograd::variable_list& grads) override;
  std::weak_ptr<Reducer> red;
  int64_t idx;
};

class Reducer : public std::enable_shared_from_this<Reducer> {
 public:
  Reducer(std::vector<at::Tensor> params, c10::intrusive_ptr<c10d::ProcessGroup> pg,
          int64_t message_size, int64_t allreduce_fp32_mode, double predivide,
          bool gradient_average, bool delay_allreduce, bool use_avg_op,
          std::vector<int64_t> trigger_params, int64_t align)
      : params_(std::move(params)),
        pg_(std::move(pg)),
        message_size_(message_size > 0 ? message_size : 1),
        fp32_mode_(allreduce_fp32_mode),
        predivide_(predivide),
        average_(gradient_average),
        delay_(delay_allreduce),
        use_avg_(use_avg_op),
        align_(align > 0 ? align : 1) {
    world_ = pg_ ? pg_->getSize() : 1;
    rank_ = pg_ ? pg_->getRank() : 0;
    for (int64_t t : trigger_params) triggers_.insert(t);
    std::vector<int64_t> order;
    for (int64_t i = (int64_t)params_.size() - 1; i >= 0; --i) order.push_back(i);
    build_layout(order);
    seen_.assign(params_.size(), 0);
    async_marked_.assign(params_.size(), 0);
    no_direct_.assign(params_.size(), 0);
    lazy_.assign(params_.size(), 0);
    side_ev_.assign(params_.size(), nullptr);
  }

  ~Reducer() {
    remove_hooks();
    if (ev_start_) {
      (void)hipEventDestroy(ev_start_);
      (void)hipEventDestroy(ev_bwd_end_);
    }
    for (auto e : ev_launch_) (void)hipEventDestroy(e);
    for (auto e : ev_done_) (void)hipEventDestroy(e);
    for (auto e : ev_pool_) (void)hipEventDestroy(e);
    for (auto& b : buckets_)
      for (auto e : b.waits) (void)hipEventDestroy(e);
    if (ev_main_) (void)hipEventDestroy(ev_main_);
  }

  void install_hooks() {
    std::weak_ptr<Reducer> weak = shared_from_this();
    for (size_t i = 0; i < params_.size(); ++i) {
      auto acc = torch::autograd::impl::grad_accumulator(params_[i]);
      TORCH_CHECK(acc, "parameter ", i, " has no grad accumulator (requires_grad=False?)");
      const int64_t idx = (int64_t)i;
      auto key = acc->add_post_hook(std::make_unique<torch::autograd::utils::LambdaPostHook>(
          [weak, idx](const torch::autograd::variable_list& outputs,
                      const torch::autograd::variable_list& inputs) {
            if (auto self = weak.lock())
              self->mark_ready_hook(idx, !inputs.empty() && inputs[0].defined());
            return outputs;
          }));
      accs_.push_back(acc);
      hook_keys_.push_back(key);
      auto pre = std::make_unique<SideWaitPreHook>(weak, idx);
      pre_keys_.push_back(pre.get());
      acc->add_pre_hook(std::move(pre));
    }
  }

  void remove_hooks() {
    for (size_t i = 0; i < accs_.size(); ++i) {
      accs_[i]->del_post_hook(hook_keys_[i]);
      auto& pres = accs_[i]->pre_hooks();
      for (auto it = pres.begin(); it != pres.end(); ++it)
        if (it->get() == pre_keys_[i]) {
          pres.erase(it);
          break;
        }
    }
    accs_.clear();
    hook_keys_.clear();
    pre_keys_.clear();
  }

  // AccumulateGrad pre-hook: a parameter whose gradient a SIDE stream wrote into its
  // bucket view (mark_ready_on_stream) and that ALSO receives an autograd gradient from
  // another use (an explicit penalty term, say): AccumulateGrad adds that gradient into
  // the same view on the compute stream, which must first wait for the side stream's
  // write.  Without another use the incoming gradient is undefined and
  // nothing waits.
  void side_wait(int64_t i, bool incoming) {
    if (!incoming) return;
    std::lock_guard<std::mutex> g(mu_);
    hipEvent_t e = side_ev_[(size_t)i];
    if (e == nullptr) return;
    TORCH_CHECK(hipStreamWaitEvent(c10::hip::getCurrentHIPStream().stream(), e, 0) == hipSuccess,
                "hipStreamWaitEvent failed");
  }

  // ---- hook path (autograd engine thread) ---------------------------------
  void mark_ready(int64_t i) { mark_ready_impl(i, nullptr); }
  // the AccumulateGrad post-hook; `had_grad`: autograd accumulated a gradient into the
  // parameter's .grad (bucket view) in this call
  void mark_ready_hook(int64_t i, bool had_grad) {
    mark_ready_impl(i, nullptr, false, true, had_grad);
  }

  // A gradient already accumulated into its bucket view by work on `stream`
  // (side-stream weight gradients): ready once that stream reaches this point.
  // announced by the caller (a side stream, or a kernel that accumulated straight into
  // the bucket view on the compute stream - which may be the null stream, handle 0)
  void mark_ready_on_stream(int64_t i, int64_t stream) {
    mark_ready_impl(i, reinterpret_cast<hipStream_t>(stream), true);
  }
  // announced from the compute stream itself (the gradient was accumulated into the
  // bucket view by a kernel on it): no event - the bucket launch already waits for the
  // compute stream
  void mark_ready_direct(int64_t i) { mark_ready_impl(i, nullptr, true, false); }

  // Side-stream gradients can be announced (iteration >= 2 of an overlapped,
  // enabled reducer whose collectives run): the caller then writes the gradient
  // into the bucket view itself and calls mark_ready_on_stream.
  bool async_ready_ok() const { return enabled_ && !refresh_ && !delay_ && comm_active(); }

  // Direct / side-stream announcements are only sound for a parameter whose ONE use per
  // iteration produces its whole gradient.  Parameters the Python wrapper found shared
  // (tied weights: listed more than once in the module tree) are excluded from the
  // start; a parameter that turns out to receive an autograd gradient on top of an
  // announced one (a functional use outside the module tree) is excluded from then on.
  void set_no_direct(const std::vector<int64_t>& idx) {
    std::lock_guard<std::mutex> g(mu_);
    for (int64_t i : idx) {
      TORCH_CHECK(i >= 0 && i < (int64_t)params_.size(), "set_no_direct: bad index");
      no_direct_[(size_t)i] = 1;
    }
  }
  bool direct_ok(int64_t i) const {
    return i >= 0 && i < (int64_t)no_direct_.size() && !no_direct_[(size_t)i];
  }
  // iterations completed (reduced backwards)
  int64_t iteration() const { return iteration_; }
  // backward passes that reached this reducer's hooks, counted under no_sync /
  // disable_allreduce too: ops/_ddp_direct.py starts a new forward-use count only
  // when a backward has completed since the last DDP forward, so several forwards
  // feeding one backward (siamese / contrastive) share one count
  int64_t backwards() const { return backwards_; }

  // Lazy zeroing (the optimizers' zero_grad on bucket-view gradients): instead of a
  // memset of the buckets, the parameters' .grad are detached from their views and the
  // views marked stale.  The next backward's first contribution then WRITES the view:
  // AccumulateGrad stores its tensor as .grad and the ready hook copies it into the view
  // (the copy replaces the add it would have run), a direct-path kernel writes the view
  // with beta = 0 (lazy_view()); a parameter without a gradient gets a zeroed view at
  // the end of backward (allow_unused) as before.  Only while the reducer will see this
  // backward through (enabled, not delay_allreduce).
  bool lazy_zero_ok() const { return enabled_ && !delay_; }
  void lazy_zero(const std::vector<int64_t>& idx) {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(lazy_zero_ok(), "lazy_zero: reducer disabled or delaying");
    for (int64_t i : idx) {
      TORCH_CHECK(i >= 0 && i < (int64_t)params_.size(), "lazy_zero: bad index");
      at::Tensor& grad = params_[(size_t)i].mutable_grad();
      if (grad.defined() && !grad.is_same(views_[(size_t)i])) {
        // a gradient that is not the view (never attached): zero it the old way
        c10::NoGradGuard ng;
        grad.zero_();
        continue;
      }
      grad = at::Tensor();
      lazy_[(size_t)i] = 1;
    }
  }
  // the stale view of a lazily zeroed parameter, for a direct-path kernel to WRITE
  // (undefined when the parameter is not lazy: accumulate into .grad instead)
  at::Tensor lazy_view(int64_t i) {
    std::lock_guard<std::mutex> g(mu_);
    if (i < 0 || i >= (int64_t)params_.size() || !lazy_[(size_t)i] ||
        params_[(size_t)i].grad().defined())
      return at::Tensor();
    return views_[(size_t)i];
  }

  void mark_ready_impl(int64_t i, hipStream_t side, bool announced = false,
                       bool with_event = true, bool had_grad = false) {
    std::lock_guard<std::mutex> g(mu_);
    if (announced && lazy_[(size_t)i] && !params_[(size_t)i].grad().defined()) {
      // a lazily zeroed parameter announced by a direct-path / side-stream kernel: that
      // kernel WROTE its view (lazy_view()), so the view becomes the gradient as it is
      params_[(size_t)i].mutable_grad() = views_[(size_t)i];
      lazy_[(size_t)i] = 0;
    }
    if (announced) {
      // The announcement only records that the gradient is in the view (and, for a
      // side stream, the event the bucket's collective must wait for).  The ready mark
      // itself is left to the AccumulateGrad post-hook, which fires once every use of
      // the parameter has been summed: a bucket can then never launch before a late
      // autograd gradient of another use lands in the same view.
      TORCH_CHECK(!async_marked_[(size_t)i] && !seen_[(size_t)i],
                  "DistributedDataParallel: parameter ", i,
                  " was announced twice in one backward pass (a module used more than once "
                  "per iteration on the direct-gradient path)");
      async_marked_[(size_t)i] = 1;
      attach_view(i);
      if (with_event && enabled_ && !refresh_ && !delay_ && comm_active()) {
        hipEvent_t e = take_event();
        TORCH_CHECK(hipEventRecord(e, side) == hipSuccess, "hipEventRecord failed");
        buckets_[(size_t)bucket_of_[(size_t)i]].waits.push_back(e);
        // (valid until this parameter's bucket launches, which needs its ready mark,
        // which comes after the AccumulateGrad pre-hook that may wait on it)
        if (side != nullptr) side_ev_[(size_t)i] = e;
      }
      return;
    }
    side_ev_[(size_t)i] = nullptr;
    if (async_marked_[(size_t)i]) {
      // the AccumulateGrad post-hook of an announced gradient (the Function returned
      // None for it; the hook still runs): the parameter is ready now
      async_marked_[(size_t)i] = 0;
      // another use accumulated an autograd gradient on top of the announced one: the
      // sum in the view is correct (the bucket has not launched), but announcing this
      // parameter is pointless work from now on
      if (had_grad) no_direct_[(size_t)i] = 1;
    }
    attach_view(i);
    if (!callback_queued_) {
      callback_queued_ = true;
      if (enabled_ && timing_) timing_record(ev_start_);
      std::weak_ptr<Reducer> weak = shared_from_this();
      torch::autograd::Engine::get_default_engine().queue_callback([weak]() {
        if (auto self = weak.lock()) self->finalize();
      });
    }
    if (!enabled_) return;
    TORCH_CHECK(!seen_[(size_t)i],
                "DistributedDataParallel: parameter ", i,
                " received a gradient twice in one backward pass; use delay_allreduce=True "
                "(or disable_allreduce()) for multiple backward passes per step");
    seen_[(size_t)i] = 1;
    if (refresh_) {
      arrival_.push_back(i);
      return;
    }
    if (delay_) return;
    Bucket& b = buckets_[(size_t)bucket_of_[(size_t)i]];
    b.pending -= 1;
    while (next_ < (int64_t)buckets_.size() && buckets_[(size_t)next_].pending == 0)
      launch(next_++);
  }

  void finalize() {
    std::lock_guard<std::mutex> g(mu_);
    callback_queued_ = false;
    ++backwards_;
    if (!enabled_) return;
    RangeGuard rg(prof_, "apex_amd::ddp_epilogue");
    const bool timed = timing_ && !refresh_ && !delay_;
    if (timed) timing_record(ev_bwd_end_);
    if (refresh_) {
      rebuild_from_arrival();
      for (size_t b = 0; b < buckets_.size(); ++b) launch((int64_t)b);
      refresh_ = false;
    } else if (delay_) {
      for (size_t b = 0; b < buckets_.size(); ++b) launch((int64_t)b);
    } else if (next_ != (int64_t)buckets_.size()) {
      std::vector<int64_t> missing;
      for (size_t i = 0; i < params_.size(); ++i)
        if (!seen_[i]) missing.push_back((int64_t)i);
      if (allow_unused_) {
        // unused parameters keep zero grads in their bucket; launch the rest in order
        for (int64_t m : missing) {
          attach_view(m);
          buckets_[(size_t)bucket_of_[(size_t)m]].pending -= 1;
        }
        while (next_ < (int64_t)buckets_.size()) launch(next_++);
      } else {
        const int64_t reduced = next_;
        // drain what was launched so no collective is left dangling
        for (auto& b : buckets_) complete(b);
        reset_iteration();
        TORCH_CHECK(false, "DistributedDataParallel epilogue: only ", reduced, " of ",
                    buckets_.size(), " buckets were reduced; ", missing.size(),
                    " parameter(s) received no gradient (first missing index ",
                    missing.empty() ? -1 : missing[0],
                    "). Pass allow_unused=True or delay_allreduce=True.");
      }
    }
    for (size_t b = 0; b < buckets_.size(); ++b) {
      complete(buckets_[b]);
      if (timed) timing_record(ev_done_[b]);
    }
    timing_valid_ = timed;
    reset_iteration();
  }

  // ---- python-facing helpers ---------------------------------------------
  void set_enabled(bool e) { enabled_ = e; }
  // tapered tail buckets on / off (rebuilds the layout in the current order)
  void set_tapered(bool t) {
    std::lock_guard<std::mutex> g(mu_);
    if (t == tapered_) return;
    tapered_ = t;
    std::vector<int64_t> order = current_order();
    build_layout(order);
    if (timing_) ensure_events();
  }
  // apex num_allreduce_streams / allreduce_communicators: bucket b goes to
  // bucket_pgs[b % n] (separate RCCL communicators -> separate streams).
  void set_bucket_process_groups(std::vector<c10::intrusive_ptr<c10d::ProcessGroup>> pgs) {
    std::lock_guard<std::mutex> g(mu_);
    bucket_pgs_ = std::move(pgs);
  }
  bool enabled() const { return enabled_; }
  void set_force_collectives(bool f) { force_ = f; }
  void set_prof(bool p) { prof_ = p; }
  bool force_collectives() const { return force_; }
  bool collectives_active() const { return comm_active(); }
  void set_timing(bool t) {
    std::lock_guard<std::mutex> g(mu_);
    timing_ = t;
    timing_valid_ = false;
    if (t) ensure_events();
  }
  // Last timed iteration: {backward_ms, tail_ms, launch_ms[b]..., done_ms[b]...}.
  // backward_ms: first gradient -> end of backward; launch_ms[b]: first
  // gradient -> bucket b handed to the process group; done_ms[b]: first
  // gradient -> the compute stream has joined bucket b's collective; tail_ms:
  // end of backward -> every collective joined (communication left exposed).
  // Blocks until the iteration's events have completed.  Empty if none.
  std::vector<double> timing() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<double> r;
    if (!timing_valid_ || buckets_.empty()) return r;
    TORCH_CHECK(hipEventSynchronize(ev_done_[buckets_.size() - 1]) == hipSuccess,
                "hipEventSynchronize failed");
    auto el = [&](hipEvent_t a, hipEvent_t b) {
      float ms = 0.f;
      TORCH_CHECK(hipEventElapsedTime(&ms, a, b) == hipSuccess, "hipEventElapsedTime failed");
      return (double)ms;
    };
    const size_t nb = buckets_.size();
    r.push_back(el(ev_start_, ev_bwd_end_));
    r.push_back(el(ev_bwd_end_, ev_done_[nb - 1]));
    for (size_t b = 0; b < nb; ++b) r.push_back(el(ev_start_, ev_launch_[b]));
    for (size_t b = 0; b < nb; ++b) r.push_back(el(ev_start_, ev_done_[b]));
    return r;
  }
  void set_allow_unused(bool a) { allow_unused_ = a; }
  void force_refresh() {
    std::lock_guard<std::mutex> g(mu_);
    refresh_ = true;
  }
  bool needs_refresh() const { return refresh_; }
  int64_t num_buckets() const { return (int64_t)buckets_.size(); }
  std::vector<std::vector<int64_t>> layout() const {
    std::vector<std::vector<int64_t>> r;
    for (auto& b : buckets_) r.push_back(b.params);
    return r;
  }
  std::vector<at::Tensor> bucket_tensors() const {
    std::vector<at::Tensor> r;
    for (auto& b : buckets_) r.push_back(b.flat);
    return r;
  }
  std::vector<int64_t> bucket_numels() const {
    std::vector<int64_t> r;
    for (auto& b : buckets_) r.push_back(b.numel);
    return r;
  }
  // Attach every parameter's grad to its bucket view (zeros for missing grads).
  void attach_all() {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < params_.size(); ++i) attach_view((int64_t)i);
  }
  // Zero every bucket in one memset per bucket (grads stay views).
  void zero_grads() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& b : buckets_) b.flat.zero_();
    for (size_t i = 0; i < params_.size(); ++i) attach_view((int64_t)i);
  }

 private:
  at::Tensor view_of(int64_t i) const { return views_[(size_t)i]; }

  void attach_view(int64_t i) {
    at::Tensor& p = params_[(size_t)i];
    at::Tensor& grad = p.mutable_grad();
    const at::Tensor& v = views_[(size_t)i];
    lazy_[(size_t)i] = 0;
    if (grad.defined() && grad.is_same(v)) return;
    c10::NoGradGuard ng;
    if (grad.defined()) v.copy_(grad);
    else v.zero_();
    grad = v;
  }

  // Tapered tail (default; no custom triggers): per dtype the buckets are cut from the
  // END of the arrival order with limits message_size/16, /8, /4, /2, then message_size,
  // so the buckets that can only launch as backward ends (the first layers' gradients
  // arrive last) are small and their all-reduce - the exposed tail - is short, while the
  // early gradients still travel in full-size buckets.  Buckets launch in the order their
  // LAST gradient arrives.
  void build_tapered(const std::vector<int64_t>& order, std::vector<Bucket>& nb) {
    std::map<at::ScalarType, std::vector<int64_t>> by_type;
    std::vector<int64_t> pos(params_.size(), 0);
    for (size_t k = 0; k < order.size(); ++k) {
      pos[(size_t)order[k]] = (int64_t)k;
      by_type[params_[(size_t)order[k]].scalar_type()].push_back(order[k]);
    }
    for (auto& kv : by_type) {
      const std::vector<int64_t>& ps = kv.second;
      std::vector<std::vector<int64_t>> groups;  // from the end of the order
      int64_t limit = std::max<int64_t>(1, message_size_ / 16), acc = 0;
      std::vector<int64_t> cur;
      for (auto it = ps.rbegin(); it != ps.rend(); ++it) {
        cur.push_back(*it);
        acc += params_[(size_t)*it].numel();
        if (acc >= limit) {
          groups.push_back(cur);
          cur.clear();
          acc = 0;
          limit = std::min<int64_t>(message_size_, limit * 2);
        }
      }
      if (!cur.empty()) groups.push_back(cur);
      for (auto g = groups.rbegin(); g != groups.rend(); ++g) {
        Bucket b;
        b.dtype = kv.first;
        for (auto it = g->rbegin(); it != g->rend(); ++it) {  // arrival order inside
          int64_t off = (b.numel + align_ - 1) / align_ * align_;
          b.params.push_back(*it);
          b.offsets.push_back(off);
          b.numel = off + params_[(size_t)*it].numel();
        }
        nb.push_back(std::move(b));
      }
    }
    std::stable_sort(nb.begin(), nb.end(), [&](const Bucket& a, const Bucket& b) {
      return pos[(size_t)a.params.back()] < pos[(size_t)b.params.back()];
    });
  }

  // Apex's rule: per dtype, close a bucket once it holds message_size elements or at an
  // allreduce trigger parameter
  void build_sized(const std::vector<int64_t>& order, std::vector<Bucket>& nb) {
    std::map<at::ScalarType, Bucket> open;
    auto close = [&](at::ScalarType t) {
      auto it = open.find(t);
      if (it == open.end() || it->second.params.empty()) return;
      nb.push_back(std::move(it->second));
      open.erase(it);
    };
    for (int64_t i : order) {
      const at::Tensor& p = params_[(size_t)i];
      at::ScalarType t = p.scalar_type();
      Bucket& b = open[t];
      b.dtype = t;
      int64_t off = (b.numel + align_ - 1) / align_ * align_;
      b.params.push_back(i);
      b.offsets.push_back(off);
      b.numel = off + p.numel();
      if (b.numel >= message_size_ || triggers_.count(i)) close(t);
    }
    // close the remaining open buckets in the order of their first parameter
    std::vector<std::pair<size_t, at::ScalarType>> rest;
    for (auto& kv : open) {
      auto pos = std::find(order.begin(), order.end(), kv.second.params.front()) - order.begin();
      rest.push_back({(size_t)pos, kv.first});
    }
    std::sort(rest.begin(), rest.end());
    for (auto& r : rest) close(r.second);
  }

  void build_layout(const std::vector<int64_t>& order) {
    std::vector<Bucket> nb;
    std::vector<int64_t> bucket_of(params_.size(), -1), offset_of(params_.size(), 0);
    if (tapered_ && triggers_.empty()) build_tapered(order, nb);
    else build_sized(order, nb);
    std::vector<at::Tensor> new_views(params_.size());
    for (size_t b = 0; b < nb.size(); ++b) {
      Bucket& B = nb[b];
      const at::Tensor& p0 = params_[(size_t)B.params[0]];
      // padded to align_ * world: the reduce-scatter / all-gather form of fp32 mode 3
      // cuts the flat buffer into world equal shards
      const int64_t unit = align_ * (int64_t)world_;
      int64_t padded = (B.numel + unit - 1) / unit * unit;
      B.flat = at::zeros({padded}, p0.options().dtype(B.dtype));
      for (size_t k = 0; k < B.params.size(); ++k) {
        int64_t i = B.params[k];
        const at::Tensor& p = params_[(size_t)i];
        bucket_of[(size_t)i] = (int64_t)b;
        offset_of[(size_t)i] = B.offsets[k];
        // same strides as the parameter (channels_last weights keep their layout)
        new_views[(size_t)i] = B.flat.as_strided(p.sizes(), p.strides(), B.offsets[k]);
      }
      B.pending = (int)B.params.size();
    }
    // migrate existing gradients into the new views
    if (!views_.empty()) {
      c10::NoGradGuard ng;
      for (size_t i = 0; i < params_.size(); ++i) {
        at::Tensor& grad = params_[i].mutable_grad();
        if (grad.defined()) {
          new_views[i].copy_(grad);
          grad = new_views[i];
        }
      }
    }
    buckets_ = std::move(nb);
    bucket_of_ = std::move(bucket_of);
    views_ = std::move(new_views);
  }

  std::vector<int64_t> current_order() const {
    std::vector<int64_t> order;
    for (const auto& b : buckets_)
      for (int64_t i : b.params) order.push_back(i);
    return order;
  }

  void rebuild_from_arrival() {
    std::vector<int64_t> order = arrival_;
    std::vector<char> in(params_.size(), 0);
    for (int64_t i : order) in[(size_t)i] = 1;
    for (int64_t i = (int64_t)params_.size() - 1; i >= 0; --i)
      if (!in[(size_t)i]) order.push_back(i);
    if (comm_active()) {
      // rank 0's order wins (apex sync_bucket_structure)
      at::Tensor t = at::tensor(order, at::TensorOptions().dtype(at::kLong));
      at::Tensor dev_t = t.to(params_[0].device());
      std::vector<at::Tensor> v{dev_t};
      c10d::BroadcastOptions opts;
      opts.rootRank = 0;
      pg_->broadcast(v, opts)->wait();
      at::Tensor back = dev_t.cpu();
      const int64_t* pp = back.data_ptr<int64_t>();
      order.assign(pp, pp + back.numel());
    }
    build_layout(order);
    arrival_.clear();
    if (timing_) ensure_events();
  }

  bool comm_active() const { return world_ > 1 || force_; }

  hipEvent_t take_event() {
    if (!ev_pool_.empty()) {
      hipEvent_t e = ev_pool_.back();
      ev_pool_.pop_back();
      return e;
    }
    hipEvent_t e;
    TORCH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess,
                "hipEventCreate failed");
    return e;
  }

  void ensure_events() {
    auto grow = [](std::vector<hipEvent_t>& v, size_t n) {
      while (v.size() < n) {
        hipEvent_t e;
        TORCH_CHECK(hipEventCreate(&e) == hipSuccess, "hipEventCreate failed");
        v.push_back(e);
      }
    };
    if (!ev_start_) {
      TORCH_CHECK(hipEventCreate(&ev_start_) == hipSuccess, "hipEventCreate failed");
      TORCH_CHECK(hipEventCreate(&ev_bwd_end_) == hipSuccess, "hipEventCreate failed");
    }
    grow(ev_launch_, buckets_.size());
    grow(ev_done_, buckets_.size());
  }

  void timing_record(hipEvent_t e) {
    if (!params_[0].is_cuda()) return;
    TORCH_CHECK(hipEventRecord(e, c10::hip::getCurrentHIPStream().stream()) == hipSuccess,
                "hipEventRecord failed");
  }

  void launch(int64_t bi) {
    Bucket& B = buckets_[(size_t)bi];
    if (B.launched) return;
    B.launched = true;
    if (!comm_active()) return;
    if (timing_ && !refresh_ && !delay_) timing_record(ev_launch_[(size_t)bi]);
    RangeGuard rg(prof_, "apex_amd::allreduce_bucket " + std::to_string(bi));
    if (!B.waits.empty() || (split_mode(B) && params_[0].is_cuda())) {
      // launch stream = compute stream's work so far + every side-stream gradient
      // of this bucket; the collective (and the fp32 up-cast) run behind it
      if (!launch_stream_)
        launch_stream_ = std::make_unique<at::hip::HIPStreamMasqueradingAsCUDA>(
            at::hip::getStreamFromPoolMasqueradingAsCUDA(true, params_[0].device().index()));
      hipStream_t ls = launch_stream_->stream();
      if (!ev_main_)
        TORCH_CHECK(hipEventCreateWithFlags(&ev_main_, hipEventDisableTiming) == hipSuccess,
                    "hipEventCreate failed");
      TORCH_CHECK(hipEventRecord(ev_main_, c10::hip::getCurrentHIPStream().stream()) == hipSuccess,
                  "hipEventRecord failed");
      TORCH_CHECK(hipStreamWaitEvent(ls, ev_main_, 0) == hipSuccess, "hipStreamWaitEvent failed");
      for (hipEvent_t e : B.waits) {
        TORCH_CHECK(hipStreamWaitEvent(ls, e, 0) == hipSuccess, "hipStreamWaitEvent failed");
        ev_pool_.push_back(e);  // reusable once recorded again (waits were enqueued)
      }
      B.waits.clear();
      at::hip::HIPStreamGuardMasqueradingAsCUDA sg(*launch_stream_);
      launch_body(B, bi);
      return;
    }
    launch_body(B, bi);
  }

  // fp32 mode 3: a bf16 bucket is reduced as an fp32 reduce-scatter (each rank's shard
  // summed in fp32 over the ring, rounded to bf16 ONCE) followed by an in-place bf16
  // all-gather, at 6 instead of 8 wire bytes per element ((n-1)/n x (4 + 2) vs
  // 2 (n-1)/n x 4).  Same precision class as the fp32 all-reduce of mode 2 (fp32 sums,
  // one rounding), but not pinned bitwise to it: RCCL may order the fp32 additions of a
  // reduce-scatter differently from an all-reduce's (tested on gloo only).
  bool split_mode(const Bucket& B) const { return fp32_mode_ == 3 && B.dtype == at::kBFloat16; }

  void launch_split(Bucket& B, int64_t bi) {
    // runs on the launch stream (launch()): the compute stream never waits for the
    // reduce-scatter; the fp32 -> bf16 shard conversion sits between the collectives
    auto& pg = (bucket_pgs_.empty()) ? pg_ : bucket_pgs_[(size_t)bi % bucket_pgs_.size()];
    const int64_t P = B.flat.numel();
    TORCH_CHECK(P % world_ == 0, "reducer: bucket not padded to the world size");
    const int64_t sh = P / world_;
    const bool avg = use_avg_ && average_ && predivide_ == 1.0;
    B.comm = B.flat.to(at::kFloat);
    B.shard = at::empty({sh}, B.comm.options());
    c10d::ReduceScatterOptions ro;
    ro.reduceOp = avg ? c10d::ReduceOp(c10d::ReduceOp::AVG) : c10d::ReduceOp(c10d::ReduceOp::SUM);
    {
      RECORD_FUNCTION("apex_amd::ddp_reduce_scatter_bucket", std::vector<c10::IValue>({B.comm}));
      pg->_reduce_scatter_base(B.shard, B.comm, ro)->wait();  // this stream waits, not the host
    }
    double factor = 1.0;
    if (!avg && average_) factor = predivide_ / (double)world_;
    if (factor != 1.0) B.shard.mul_(factor);
    at::Tensor mine = B.flat.narrow(0, (int64_t)rank_ * sh, sh);
    mine.copy_(B.shard);  // the single rounding to bf16
    RECORD_FUNCTION("apex_amd::ddp_all_gather_bucket", std::vector<c10::IValue>({B.flat}));
    B.work = pg->_allgather_base(B.flat, mine);  // in place: rank r's shard is its slot
    B.split = true;
  }

  void launch_body(Bucket& B, int64_t bi) {
    c10::NoGradGuard ng;
    if (predivide_ != 1.0) B.flat.mul_(1.0 / predivide_);
    if (split_mode(B)) {
      launch_split(B, bi);
      return;
    }
    // fp32 accumulation: 1 = every 16-bit bucket (apex allreduce_always_fp32),
    // 2 = bf16 buckets only (8-bit mantissa: summing 8 ranks in bf16 rounds at
    // every ring hop).  The fp32 copy is a transient caching-allocator block
    // (recorded on the communicator's stream), not a persistent second bucket.
    const bool up = B.dtype != at::kFloat &&
                    (fp32_mode_ == 1 || (fp32_mode_ == 2 && B.dtype == at::kBFloat16));
    B.comm = up ? B.flat.to(at::kFloat) : B.flat;
    c10d::AllreduceOptions opts;
    const bool avg = use_avg_ && average_ && predivide_ == 1.0;
    opts.reduceOp = avg ? c10d::ReduceOp(c10d::ReduceOp::AVG) : c10d::ReduceOp(c10d::ReduceOp::SUM);
    std::vector<at::Tensor> v{B.comm};
    RECORD_FUNCTION("apex_amd::ddp_allreduce_bucket", std::vector<c10::IValue>({B.comm}));
    auto& pg = (bucket_pgs_.empty()) ? pg_ : bucket_pgs_[(size_t)bi % bucket_pgs_.size()];
    B.work = pg->allreduce(v, opts);
  }

  void complete(Bucket& B) {
    for (hipEvent_t e : B.waits) {  // announced but never launched (error paths)
      (void)hipStreamWaitEvent(c10::hip::getCurrentHIPStream().stream(), e, 0);
      ev_pool_.push_back(e);
    }
    B.waits.clear();
    if (!B.launched || !comm_active()) return;
    if (B.work) B.work->wait();
    c10::NoGradGuard ng;
    if (B.split) {  // averaged and rounded before the all-gather
      B.split = false;
      B.work.reset();
      B.comm = at::Tensor();
      B.shard = at::Tensor();
      return;
    }
    const bool avg = use_avg_ && average_ && predivide_ == 1.0;
    double factor = 1.0;
    if (!avg && average_) factor = predivide_ / (double)world_;
    if (!B.comm.is_same(B.flat)) {
      if (factor != 1.0) B.flat.copy_(B.comm.mul_(factor));
      else B.flat.copy_(B.comm);
    } else if (factor != 1.0) {
      B.flat.mul_(factor);
    }
    B.work.reset();
    B.comm = at::Tensor();
  }

  void reset_iteration() {
    std::fill(side_ev_.begin(), side_ev_.end(), nullptr);
    for (auto& b : buckets_) {
      b.pending = (int)b.params.size();
      b.launched = false;
      b.work.reset();
    }
    next_ = 0;
    std::fill(seen_.begin(), seen_.end(), 0);
    std::fill(async_marked_.begin(), async_marked_.end(), 0);
    ++iteration_;
  }

  std::vector<at::Tensor> params_;
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  std::vector<c10::intrusive_ptr<c10d::ProcessGroup>> bucket_pgs_;
  int64_t message_size_;
  int64_t fp32_mode_;
  double predivide_;
  bool average_, delay_, use_avg_;
  int64_t align_;
  int world_ = 1, rank_ = 0;
  std::set<int64_t> triggers_;

  std::vector<Bucket> buckets_;
  std::vector<int64_t> bucket_of_;
  std::vector<at::Tensor> views_;
  std::vector<int64_t> arrival_;
  std::vector<char> seen_;
  std::vector<char> async_marked_;
  std::vector<char> no_direct_;
  std::vector<char> lazy_;
  int64_t iteration_ = 0;
  int64_t backwards_ = 0;
  bool tapered_ = true;
  int64_t next_ = 0;
  bool refresh_ = true;
  bool enabled_ = true;
  bool allow_unused_ = false;
  bool callback_queued_ = false;
  bool force_ = false;
  bool timing_ = false, timing_valid_ = false;
  bool prof_ = false;
  std::vector<hipEvent_t> ev_pool_;
  std::vector<hipEvent_t> side_ev_;  // per parameter: its side-stream announcement event
  std::vector<torch::autograd::FunctionPreHook*> pre_keys_;
  hipEvent_t ev_main_ = nullptr;
  std::unique_ptr<at::hip::HIPStreamMasqueradingAsCUDA> launch_stream_;
  hipEvent_t ev_start_ = nullptr, ev_bwd_end_ = nullptr;
  std::vector<hipEvent_t> ev_launch_, ev_done_;
  std::mutex mu_;

  std::vector<std::shared_ptr<torch::autograd::Node>> accs_;
  std::vector<uintptr_t> hook_keys_;
};

torch::autograd::variable_list SideWaitPreHook::operator()(
    const torch::autograd::variable_list& grads) {
  if (auto r = red.lock()) r->side_wait(idx, !grads.empty() && grads[0].defined());
  return grads;
}

std::shared_ptr<Reducer> make_reducer(std::vector<at::Tensor> params,
                                      c10::intrusive_ptr<c10d::ProcessGroup> pg,
                                      int64_t message_size, int64_t allreduce_fp32_mode,
                                      double predivide, bool gradient_average,
                                      bool delay_allreduce, bool use_avg_op,
                                      std::vector<int64_t> trigger_params, int64_t align) {
  auto r = std::make_shared<Reducer>(std::move(params), std::move(pg), message_size,
                                     allreduce_fp32_mode, predivide, gradient_average,
                                     delay_allreduce, use_avg_op, std::move(trigger_params), align);
  r->install_hooks();
  return r;
}

}  // namespace

// ---- SyncBatchNorm collectives from C++ (ops/batch_norm.py's RCCL path): one call per
// BN layer instead of the Python c10d wrappers (~20 us of host time each, 2 per layer
// per step: ResNet-50 went host-bound at world 1 with forced collectives).
std::tuple<at::Tensor, at::Tensor, at::Tensor> syncbn_allgather_combine(
    at::Tensor packed, c10::intrusive_ptr<c10d::ProcessGroup> pg, double eps, double momentum,
    c10::optional<at::Tensor> running_mean, c10::optional<at::Tensor> running_var,
    c10::optional<at::Tensor> nbt) {
  c10::NoGradGuard ng;
  TORCH_CHECK(packed.is_cuda() && packed.is_contiguous(), "syncbn: packed stats on the GPU");
  const int world = pg->getSize();
  at::Tensor gathered = at::empty({world * packed.numel()}, packed.options());
  pg->_allgather_base(gathered, packed)->wait();  // stream-ordered for RCCL (no host block)
  return bn_combine_stats_sync_op(gathered.view({world, -1}), eps, momentum, running_mean,
                                  running_var, nbt);
}

void syncbn_allreduce(at::Tensor t, c10::intrusive_ptr<c10d::ProcessGroup> pg) {
  c10::NoGradGuard ng;
  std::vector<at::Tensor> ts{t};
  pg->allreduce(ts)->wait();
}

// ---- the same collectives issued on the COMPUTE stream through the SyncBN group's own
// RCCL communicator (ProcessGroupNCCL._comm_ptr()): no hand-off to the process group's
// stream and back (two cross-stream event waits per call, ~20 us of bubble each; ResNet-50
// runs 106 of them per step).  Safe because that communicator is used by SyncBN only and
// every SyncBN collective is stream-ordered on the compute stream (never two in flight).
// The functions are looked up in the RCCL that torch itself loaded (RTLD_DEFAULT), so the
// communicator and the calls come from one library.
namespace {
using AllGatherFn = ncclResult_t (*)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                                     hipStream_t);
using AllReduceFn = ncclResult_t (*)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t,
                                     ncclComm_t, hipStream_t);
AllGatherFn rccl_allgather() {
  static AllGatherFn f = reinterpret_cast<AllGatherFn>(dlsym(RTLD_DEFAULT, "ncclAllGather"));
  return f;
}
AllReduceFn rccl_allreduce() {
  static AllReduceFn f = reinterpret_cast<AllReduceFn>(dlsym(RTLD_DEFAULT, "ncclAllReduce"));
  return f;
}
}  // namespace

bool syncbn_raw_available() { return rccl_allgather() && rccl_allreduce(); }

// The rank count and this process's rank as the RCCL communicator itself reports them
// (bench.py records them at N > 1: what the collectives really span).
std::tuple<int64_t, int64_t> rccl_comm_info(int64_t comm) {
  using CountFn = ncclResult_t (*)(const ncclComm_t, int*);
  static CountFn count = reinterpret_cast<CountFn>(dlsym(RTLD_DEFAULT, "ncclCommCount"));
  static CountFn urank = reinterpret_cast<CountFn>(dlsym(RTLD_DEFAULT, "ncclCommUserRank"));
  TORCH_CHECK(count && urank, "rccl_comm_info: RCCL entry points not found");
  TORCH_CHECK(comm != 0, "rccl_comm_info: no communicator");
  int n = -1, r = -1;
  TORCH_CHECK(count(reinterpret_cast<ncclComm_t>(comm), &n) == ncclSuccess, "ncclCommCount failed");
  TORCH_CHECK(urank(reinterpret_cast<ncclComm_t>(comm), &r) == ncclSuccess,
              "ncclCommUserRank failed");
  return {n, r};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> syncbn_allgather_combine_raw(
    at::Tensor packed, int64_t comm, int64_t world, double eps, double momentum,
    c10::optional<at::Tensor> running_mean, c10::optional<at::Tensor> running_var,
    c10::optional<at::Tensor> nbt, c10::optional<at::Tensor> gathered_in, int64_t rank) {
  c10::NoGradGuard ng;
  TORCH_CHECK(syncbn_raw_available(), "syncbn: RCCL entry points not found");
  TORCH_CHECK(comm != 0 && world >= 1, "syncbn: no communicator");
  TORCH_CHECK(packed.is_cuda() && packed.is_contiguous() && packed.scalar_type() == at::kFloat,
              "syncbn: packed fp32 stats on the GPU");
  at::Tensor gathered;
  if (gathered_in.has_value() && gathered_in->defined()) {
    // in-place gather: the stats kernels wrote this rank's slot of the destination
    // (RCCL skips the send-buffer copy; at world 1 the collective is a no-op)
    gathered = *gathered_in;
    TORCH_CHECK(gathered.is_contiguous() && gathered.scalar_type() == at::kFloat &&
                    gathered.numel() == world * packed.numel() && rank >= 0 && rank < world &&
                    packed.data_ptr<float>() == gathered.data_ptr<float>() + rank * packed.numel(),
                "syncbn: packed must be rank's slot of gathered");
  } else {
    gathered = at::empty({world * packed.numel()}, packed.options());
  }
  const ncclResult_t r = rccl_allgather()(packed.data_ptr(), gathered.data_ptr(),
                                          (size_t)packed.numel(), ncclFloat32,
                                          reinterpret_cast<ncclComm_t>(comm),
                                          c10::hip::getCurrentHIPStream().stream());
  TORCH_CHECK(r == ncclSuccess, "syncbn: ncclAllGather failed (", (int)r, ")");
  return bn_combine_stats_sync_op(gathered.view({world, -1}), eps, momentum, running_mean,
                                  running_var, nbt);
}

void syncbn_allreduce_raw(at::Tensor t, int64_t comm) {
  c10::NoGradGuard ng;
  TORCH_CHECK(syncbn_raw_available(), "syncbn: RCCL entry points not found");
  TORCH_CHECK(comm != 0, "syncbn: no communicator");
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat, "syncbn: fp32 GPU tensor");
  const ncclResult_t r = rccl_allreduce()(t.data_ptr(), t.data_ptr(), (size_t)t.numel(),
                                          ncclFloat32, ncclSum, reinterpret_cast<ncclComm_t>(comm),
                                          c10::hip::getCurrentHIPStream().stream());
  TORCH_CHECK(r == ncclSuccess, "syncbn: ncclAllReduce failed (", (int)r, ")");
}

// ---- side-stream gradients outside DDP (ops/conv.py _SideWgrad 'free' mode) --------
// A weight gradient computed on the side stream is stored as the parameter's .grad
// directly (autograd gets None).  If the parameter has another use whose autograd
// gradient reaches its AccumulateGrad node (an explicit penalty, a second call of the
// module), AccumulateGrad adds it into that .grad on the compute stream: this
// pre-hook makes the compute stream wait for the side stream's write first.  One hook
// (with its own event) per AccumulateGrad node, installed on first use.
namespace {
struct SideGradWait : torch::autograd::FunctionPreHook {
  hipEvent_t ev = nullptr;
  bool pending = false;
  ~SideGradWait() override {
    if (ev) (void)hipEventDestroy(ev);
  }
  torch::autograd::variable_list operator()(const torch::autograd::variable_list& grads) override {
    if (pending) {
      pending = false;
      if (!grads.empty() && grads[0].defined())
        TORCH_CHECK(hipStreamWaitEvent(c10::hip::getCurrentHIPStream().stream(), ev, 0) ==
                        hipSuccess, "hipStreamWaitEvent failed");
    }
    return grads;
  }
};
}  // namespace

void side_grad_announce(const at::Tensor& param, int64_t stream) {
  auto acc = torch::autograd::impl::grad_accumulator(param);
  TORCH_CHECK(acc, "side_grad_announce: parameter has no grad accumulator");
  SideGradWait* h = nullptr;
  for (auto& ph : acc->pre_hooks())
    if ((h = dynamic_cast<SideGradWait*>(ph.get())) != nullptr) break;
  if (h == nullptr) {
    auto u = std::make_unique<SideGradWait>();
    TORCH_CHECK(hipEventCreateWithFlags(&u->ev, hipEventDisableTiming) == hipSuccess,
                "hipEventCreateWithFlags failed");
    h = u.get();
    acc->add_pre_hook(std::move(u));
  }
  TORCH_CHECK(hipEventRecord(h->ev, reinterpret_cast<hipStream_t>(stream)) == hipSuccess,
              "hipEventRecord failed");
  h->pending = true;
}

void register_reducer(pybind11::module_& m) {
  m.def("side_grad_announce", &side_grad_announce, py::arg("param"), py::arg("stream"));
  namespace py = pybind11;
  m.def("syncbn_raw_available", &syncbn_raw_available);
  m.def("rccl_comm_info", &rccl_comm_info, py::arg("comm"));
  m.def("syncbn_allgather_combine_raw", &syncbn_allgather_combine_raw, py::arg("packed"),
        py::arg("comm"), py::arg("world"), py::arg("eps"), py::arg("momentum"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("nbt") = py::none(),
        py::arg("gathered") = py::none(), py::arg("rank") = -1);
  m.def("syncbn_allreduce_raw", &syncbn_allreduce_raw, py::arg("t"), py::arg("comm"));
  m.def("syncbn_allgather_combine", &syncbn_allgather_combine, py::arg("packed"), py::arg("pg"),
        py::arg("eps"), py::arg("momentum"), py::arg("running_mean"), py::arg("running_var"),
        py::arg("nbt") = py::none());
  m.def("syncbn_allreduce", &syncbn_allreduce, py::arg("t"), py::arg("pg"));
  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init(&make_reducer), py::arg("params"), py::arg("process_group"),
           py::arg("message_size") = 10000000, py::arg("allreduce_fp32_mode") = 0,
           py::arg("gradient_predivide_factor") = 1.0, py::arg("gradient_average") = true,
           py::arg("delay_allreduce") = false, py::arg("use_avg_op") = true,
           py::arg("trigger_params") = std::vector<int64_t>{}, py::arg("align") = 64)
      .def("set_enabled", &Reducer::set_enabled)
      .def("set_bucket_process_groups", &Reducer::set_bucket_process_groups)
      .def("enabled", &Reducer::enabled)
      .def("set_allow_unused", &Reducer::set_allow_unused)
      .def("set_force_collectives", &Reducer::set_force_collectives)
      .def("set_prof", &Reducer::set_prof)
      .def("mark_ready_on_stream", &Reducer::mark_ready_on_stream, py::arg("index"),
           py::arg("stream"))
      .def("async_ready_ok", &Reducer::async_ready_ok)
      .def("mark_ready_direct", &Reducer::mark_ready_direct)
      .def("set_no_direct", &Reducer::set_no_direct)
      .def("set_tapered", &Reducer::set_tapered)
      .def("lazy_zero_ok", &Reducer::lazy_zero_ok)
      .def("lazy_zero", &Reducer::lazy_zero)
      .def("lazy_view", &Reducer::lazy_view)
      .def("direct_ok", &Reducer::direct_ok)
      .def("iteration", &Reducer::iteration)
      .def("backwards", &Reducer::backwards)
      .def("force_collectives", &Reducer::force_collectives)
      .def("collectives_active", &Reducer::collectives_active)
      .def("set_timing", &Reducer::set_timing)
      .def("timing", &Reducer::timing)
      .def("force_refresh", &Reducer::force_refresh)
      .def("needs_refresh", &Reducer::needs_refresh)
      .def("num_buckets", &Reducer::num_buckets)
      .def("layout", &Reducer::layout)
      .def("bucket_tensors", &Reducer::bucket_tensors)
      .def("bucket_numels", &Reducer::bucket_numels)
      .def("attach_all", &Reducer::attach_all)
      .def("zero_grads", &Reducer::zero_grads)
      .def("remove_hooks", &Reducer::remove_hooks);
}

}  // namespace amd
