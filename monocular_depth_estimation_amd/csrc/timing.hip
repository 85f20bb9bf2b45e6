// Opt-in per-kernel timing registry behind mde_timing_* (include/mde_abi.h).
// Each timed launch is bracketed by two hipEvents recorded on the launch
// stream; mde_timing_collect() resolves them into per-kernel totals.
// A launch made while its stream is being captured into a hipGraph records
// its events as external event-record nodes (hipEventRecordExternal): every
// replay of that graph re-records them, and mde_timing_collect() accumulates
// the last replay's times while keeping those events for the next replay —
// per-kernel times of the REPLAYED step (collect once after each replay).
#include <mutex>
#include <vector>

#include "common.h"

namespace {

const char* const kNames[mde::K_COUNT] = {
    "bilinear_fwd",  "bilinear_bwd",    "nearest_fwd",   "nearest_bwd",
    "se_squeeze",    "se_fc",           "se_scale",      "se_bwd_dot",
    "se_bwd_fc",     "se_bwd_apply",    "skip_reduce_fwd", "skip_reduce_bwd",
    "skip_reduce_bwd_reduce", "minmax", "minmax_final", "depthnorm_apply",
    "ssim3_l1",      "loss_final",      "depth_loss_fwd", "depth_loss_bwd_coef",
    "depth_loss_bwd", "bn_fwd_stats",  "bn_fwd_final",  "bn_fwd_apply",
    "bn_bwd_reduce",  "bn_bwd_final",  "bn_bwd_apply",  "bn_fwd_apply_small",
    "bn_bwd_apply_small", "window_attn_fwd", "window_attn_bwd",
    "dwconv_fwd",    "dwconv_bwd_data", "dwconv_bwd_weight", "dwconv_wreduce",
    "layernorm_fwd", "layernorm_bwd",   "layernorm_wreduce", "transpose",
    "pointwise_fwd", "pointwise_bwd", "conv3x3_fwd",  "conv3x3_dgrad",
    "conv3x3_wgrad", "conv3x3_wreduce", "dwconv_bwd", "eval_sums", "eval_final", "nyu_augment",
    "conv3x3_wgrad_guide", "linear_bias_grad", "gelu_bwd_bias_grad", "conv3x3_fwd_bf16",
    "conv3x3_dgrad_bf16", "conv3x3_wgrad_bf16", "conv3x3_wgrad_wide", "conv3x3s2_wgrad",
    "conv1x1_fwd",   "conv1x1_dgrad",   "conv1x1_wgrad", "conv1x1_wreduce",
    "conv3x3s2_fwd", "conv3x3s2_dgrad", "conv3x3w_fwd", "conv3x3w_dgrad",
    "wino_fwd",       "wino_dgrad",      "wino_weight",   "window_attn_bwd_reduce",
    "convbf_fwd_bf16", "convbf_dgrad_bf16", "convbf_wgrad_bf16", "convbf_wreduce", "convbf_pack",
    "stem_fwd_bf16", "stem_wgrad_bf16", "linear_wgrad", "linear_wreduce", "conv_bias_grad",
    "head_conv_fwd", "head_conv_dgrad", "head_conv_wgrad"};

struct Pending {
  int kid;
  hipEvent_t a, b;
  double bytes, flops;
  bool done;
  bool captured;  // recorded inside a graph capture: kept across collects
};

struct Registry {
  std::mutex mu;
  bool on = false;
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
  double ms[mde::K_COUNT] = {};
  int64_t launches[mde::K_COUNT] = {};
  double bytes[mde::K_COUNT] = {};
  double flops[mde::K_COUNT] = {};

  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
};

Registry& reg() {
  static Registry r;
  return r;
}

// Record `e` on `s`.  Inside a capture: as an external event node
// (hipEventRecordExternal), else by adding an event-record node to the
// capturing graph by hand and making it the stream's capture dependency.
// Errors are cleared so that they never reach the kernel launch's
// hipGetLastError check.
bool record(hipEvent_t e, hipStream_t s, bool captured) {
  if (!captured) {
    const bool ok = hipEventRecord(e, s) == hipSuccess;
    if (!ok) (void)hipGetLastError();
    return ok;
  }
  if (hipEventRecordWithFlags(e, s, hipEventRecordExternal) == hipSuccess) return true;
  (void)hipGetLastError();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  hipGraphNode_t node = nullptr;
  bool ok = hipStreamGetCaptureInfo_v2(s, &cs, &id, &g, &deps, &nd) == hipSuccess && g &&
            hipGraphAddEventRecordNode(&node, g, deps, nd, e) == hipSuccess &&
            hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies) ==
                hipSuccess;
  if (!ok) (void)hipGetLastError();
  return ok;
}

}  // namespace

namespace mde {

int timing_begin(int kid, hipStream_t s) {
  Registry& r = reg();
  if (!r.on) return -1;
  std::lock_guard<std::mutex> g(r.mu);
  Pending p{kid, r.get(), r.get(), 0.0, 0.0, false, false};
  if (!p.a || !p.b) return -1;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(s, &cs);
  p.captured = cs == hipStreamCaptureStatusActive;
  if (!record(p.a, s, p.captured)) {
    r.pool.push_back(p.a);
    r.pool.push_back(p.b);
    return -1;
  }
  r.pending.push_back(p);
  return (int)r.pending.size() - 1;
}

void timing_end(int token, hipStream_t s, double bytes, double flops) {
  if (token < 0) return;
  Registry& r = reg();
  std::lock_guard<std::mutex> g(r.mu);
  if (token >= (int)r.pending.size()) return;
  Pending& p = r.pending[token];
  p.bytes = bytes;
  p.flops = flops;
  p.done = record(p.b, s, p.captured);
}

}  // namespace mde

extern "C" {

int mde_timing_enable(int on) {
  reg().on = on != 0;
  return MDE_OK;
}

int mde_timing_reset(void) {
  Registry& r = reg();
  std::lock_guard<std::mutex> g(r.mu);
  for (auto& p : r.pending) {
    r.pool.push_back(p.a);
    r.pool.push_back(p.b);
  }
  r.pending.clear();
  for (int k = 0; k < mde::K_COUNT; ++k) {
    r.ms[k] = 0.0;
    r.launches[k] = 0;
    r.bytes[k] = 0.0;
    r.flops[k] = 0.0;
  }
  return MDE_OK;
}

int mde_timing_collect(void) {
  Registry& r = reg();
  std::lock_guard<std::mutex> g(r.mu);
  int status = MDE_OK;
  std::vector<Pending> keep;
  for (auto& p : r.pending) {
    if (p.done) {
      hipError_t e = hipEventSynchronize(p.b);
      float t = 0.f;
      if (e == hipSuccess) e = hipEventElapsedTime(&t, p.a, p.b);
      if (e == hipSuccess) {
        r.ms[p.kid] += t;
        r.launches[p.kid] += 1;
        r.bytes[p.kid] += p.bytes;
        r.flops[p.kid] += p.flops;
      } else {
        status = (int)e;
      }
    }
    if (p.captured) {
      keep.push_back(p);
      continue;
    }
    r.pool.push_back(p.a);
    r.pool.push_back(p.b);
  }
  r.pending.swap(keep);
  return status;
}

int mde_kernel_count(void) { return mde::K_COUNT; }

const char* mde_kernel_name(int kid) {
  if (kid < 0 || kid >= mde::K_COUNT) return "";
  return kNames[kid];
}

int mde_timing_query(int kid, double* total_ms, int64_t* launches,
                     double* bytes) {
  if (kid < 0 || kid >= mde::K_COUNT) return MDE_ERR_INVALID_ARG;
  Registry& r = reg();
  std::lock_guard<std::mutex> g(r.mu);
  if (total_ms) *total_ms = r.ms[kid];
  if (launches) *launches = r.launches[kid];
  if (bytes) *bytes = r.bytes[kid];
  return MDE_OK;
}

int mde_timing_query_flops(int kid, double* flops) {
  if (kid < 0 || kid >= mde::K_COUNT || !flops) return MDE_ERR_INVALID_ARG;
  Registry& r = reg();
  std::lock_guard<std::mutex> g(r.mu);
  *flops = r.flops[kid];
  return MDE_OK;
}

int mde_abi_version(void) { return MDE_ABI_VERSION; }

const char* mde_status_string(int status) {
  if (status == MDE_OK) return "ok";
  if (status == MDE_ERR_INVALID_ARG) return "mde: invalid argument";
  if (status == MDE_ERR_UNSUPPORTED) return "mde: unsupported dtype/shape";
  if (status > 0) return hipGetErrorString((hipError_t)status);
  return "mde: unknown status";
}

}  // extern "C"
