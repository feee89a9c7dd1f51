// Warm-step plan: one density-weighted AL iteration (dal_dw_step) captured
// once as a hipGraph over caller-owned static buffers and replayed by
// dal_dw_plan_run.  The per-step refresh (stamp the unlabeled rows, whose list
// address and length are the mark kernel's arguments, rewritten per replay;
// the score kernel builds the step's row flags from the base flags and the
// stamps) runs inside the graph; the graph's last kernel writes the
// selection into the caller's fresh buffer and the status word into
// host-mapped memory -- the host side of a warm step is ONE call, and the
// host spins on that word instead of a blocking stream sync.
//
// Reference: the body of density_weighting.py:133-176 (per iteration: T x
// predict, entropy x density, sortBy, take(window_size)) with the proximity
// matrix of :58-100 cached across iterations, as the reference does.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <new>

#include "common.hpp"

// Host-mapped words the graph's last kernel publishes into: the selection's
// destination (a fresh tensor each step, set by the host before the replay)
// and the final status word.  No copy launches follow the graph.
struct PlanSlot {
  int64_t* out[2];     // selected indices (int64 [k]), selected scores (fp64 [k])
  int32_t status;
};

namespace {

constexpr int kPlanThreads = 256;

// In-graph row marking: stamp[r] = step for every listed row of this pool;
// the score kernel ORs DAL_ROW_CANDIDATE into the base flags where stamp[r] ==
// step (no per-step copy of the flags).  The list's (address, length) and the
// step id are kernel arguments, rewritten before each replay by
// hipGraphExecKernelNodeSetParams: no host-memory reads in the graph.  Block 0
// publishes the step id for the score kernel.  Stamps are 8-bit (a quarter of
// the bytes to write, and to write back from L2 before the score kernel):
// step ids cycle through 1..255 and dal_dw_plan_run clears the stamps when
// they wrap.  Four list entries per thread are loaded before their stores;
// the grid (fixed at capture: the list length varies per iteration) covers a
// list as long as the pool in one pass, so every load is in flight at once
// (512 blocks looping over config 4's 2M rows: 9.8 us in the step).
constexpr int kMarkPer = 4;
#ifndef DAL_PLAN_MARK_BLOCKS
#define DAL_PLAN_MARK_BLOCKS 0  // > 0: a fixed grid (rounds 3-5: 512)
#endif
inline unsigned mark_grid(int64_t n) {
  const int64_t g = DAL_PLAN_MARK_BLOCKS > 0 ? DAL_PLAN_MARK_BLOCKS
                                             : dal::ceil_div(n, static_cast<int64_t>(kPlanThreads) * kMarkPer);
  return static_cast<unsigned>(g < 1 ? 1 : g > 65535 ? 65535 : g);
}
__global__ __launch_bounds__(kPlanThreads) void plan_mark_direct_kernel(const int64_t* __restrict__ idx, int64_t count,
                                                                        uint32_t step, int64_t row_base, int64_t n,
                                                                        uint8_t* __restrict__ stamp,
                                                                        uint32_t* __restrict__ step_dev) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *step_dev = step;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kPlanThreads * kMarkPer;
  for (int64_t t0 = static_cast<int64_t>(blockIdx.x) * kPlanThreads * kMarkPer + threadIdx.x; t0 < count;
       t0 += stride) {
    int64_t r[kMarkPer];
#pragma unroll
    for (int j = 0; j < kMarkPer; ++j) {
      const int64_t t = t0 + j * kPlanThreads;
      r[j] = t < count ? idx[t] - row_base : -1;
    }
#pragma unroll
    for (int j = 0; j < kMarkPer; ++j)
      if (r[j] >= 0 && r[j] < n) stamp[r[j]] = static_cast<uint8_t>(step);
  }
}

// The step id of the plan's n-th replay: 1..255, cycling (8-bit stamps).
inline uint32_t stamp_step(uint32_t step) { return (step - 1u) % 255u + 1u; }

}  // namespace

struct dal_dw_plan {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  const uint8_t* base_flags = nullptr;
  uint8_t* flags = nullptr;
  int64_t n = 0, row_base = 0, k = 0;
  const int64_t* out_pair = nullptr;  // device [2k]: selected indices | selected score bits
  int32_t* dev_status = nullptr;
  PlanSlot* slot = nullptr;       // host view
  PlanSlot* slot_dev = nullptr;   // the same words as the device addresses them
  uint8_t* stamp = nullptr;       // device: n per-row 8-bit mark stamps, then (4-B aligned) the step id
  uint32_t* step_dev = nullptr;   // the step id word after the stamps
  int device = 0;                 // the HIP device of the capture stream (every call runs there)
  hipGraphNode_t mark_node = nullptr;  // the mark kernel's node (its arguments change every replay)
  hipKernelNodeParams mark_params{};   // its launch shape, reused by every SetParams
  uint32_t step = 0;
};

using namespace dal;

// Makes the device of ``stream`` current for the guard's lifetime (and
// restores the caller's): the plan's allocations, capture stream and graph
// must live on the device whose buffers the captured kernels read, whichever
// device the calling thread has current.
class DeviceGuard {
 public:
  explicit DeviceGuard(hipStream_t st) {
    if (hipGetDevice(&prev_) != hipSuccess) return;
    hipDevice_t dev = prev_;
    if (st && hipStreamGetDevice(st, &dev) != hipSuccess) return;
    dev_ = dev;
    ok_ = dev == prev_ || hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (ok_ && dev_ != prev_) (void)hipSetDevice(prev_);
  }
  bool ok() const { return ok_; }
  int device() const { return dev_; }

 private:
  int prev_ = 0, dev_ = 0;
  bool ok_ = false;
};

extern "C" int dal_dw_plan_create(const float* x, const float* xb, const void* fprep, int64_t n, int64_t d,
                                  int64_t ldx,
                                  const int32_t* inner,
                                  const uint8_t* leaf, int32_t n_trees, int32_t depth, const double* lut,
                                  const int64_t* density_fixed, double density_err, const uint8_t* base_flags,
                                  uint8_t* flags, double beta, int64_t idx_base, const double* norm64,
                                  const double* colsum, int64_t k, int64_t cap, int32_t level1_passes, void* ws,
                                  size_t ws_bytes, int32_t* votes, double* scores, uint64_t* keys_lo,
                                  uint64_t* keys_hi, int64_t* out_pair, uint64_t* out_keys, int32_t* dev_status,
                                  dal_stream_t stream, dal_dw_plan_t** plan_out) {
  if (!plan_out || !base_flags || !flags || !out_pair || !ws) return DAL_ERR_ARG;
  *plan_out = nullptr;
  if (n < 1 || k < 1) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  const DeviceGuard guard(st);
  if (!guard.ok()) return DAL_ERR_HIP;
  // the fused step leaves its level-1 header zero after every replay: zero it once
  if (hipMemsetAsync(ws, 0, ws_bytes, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
    return DAL_ERR_HIP;
  dal_dw_plan* p = new (std::nothrow) dal_dw_plan;
  if (!p) return DAL_ERR_HIP;
  p->device = guard.device();
  hipStream_t cs = nullptr;
  int rc = DAL_OK;
  if (hipHostMalloc(reinterpret_cast<void**>(&p->slot), sizeof(PlanSlot), hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&p->slot_dev), p->slot, 0) != hipSuccess)
    rc = DAL_ERR_HIP;
  if (!rc) {
    p->slot->out[0] = p->slot->out[1] = nullptr;
    p->slot->status = 0;
  }
  // stamps start at 0 and steps at 1: no row is marked before its first step
  const size_t stamp_bytes = static_cast<size_t>(round_up(n, 4)) + sizeof(uint32_t);
  if (!rc && (hipMalloc(reinterpret_cast<void**>(&p->stamp), stamp_bytes) != hipSuccess ||
              hipMemsetAsync(p->stamp, 0, stamp_bytes, st) != hipSuccess ||
              hipStreamSynchronize(st) != hipSuccess))
    rc = DAL_ERR_HIP;
  if (!rc) p->step_dev = reinterpret_cast<uint32_t*>(p->stamp + round_up(n, 4));
  if (!rc && hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) rc = DAL_ERR_HIP;
  if (!rc && hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) != hipSuccess) rc = DAL_ERR_HIP;
  if (!rc) {
    hipLaunchKernelGGL(plan_mark_direct_kernel, dim3(mark_grid(n)), dim3(kPlanThreads), 0, cs,
                       static_cast<const int64_t*>(nullptr), int64_t{0}, 0u, idx_base, n, p->stamp, p->step_dev);
    ForestStepHooks hooks;
    hooks.base_flags = base_flags;
    hooks.stamp = p->stamp;
    hooks.step_id = p->step_dev;
    const int step_rc = dw_step_impl(x, xb, fprep, n, d, ldx, inner, leaf, n_trees, depth, lut, density_fixed, density_err,
                                     flags, beta, idx_base, norm64, colsum, k, cap, level1_passes,
                                     DAL_STEP_RESET_STATUS | DAL_STEP_WS_CLEAN, ws, ws_bytes, votes, scores, keys_lo,
                                     keys_hi, out_pair, reinterpret_cast<double*>(out_pair + k), out_keys,
                                     dev_status, nullptr, cs, p->slot_dev->out, &p->slot_dev->status, &hooks);
    const hipError_t end = hipStreamEndCapture(cs, &p->graph);
    rc = step_rc ? step_rc : (end != hipSuccess ? DAL_ERR_HIP : DAL_OK);
  }
  if (!rc && hipGraphInstantiate(&p->exec, p->graph, nullptr, nullptr, 0) != hipSuccess) rc = DAL_ERR_HIP;
  if (!rc) {
    // find the mark kernel's node: its arguments change every replay
    size_t n_nodes = 0;
    hipGraphNode_t nodes[64];
    if (hipGraphGetNodes(p->graph, nullptr, &n_nodes) == hipSuccess && n_nodes <= 64 &&
        hipGraphGetNodes(p->graph, nodes, &n_nodes) == hipSuccess) {
      for (size_t i = 0; i < n_nodes && !p->mark_node; ++i) {
        hipGraphNodeType ty;
        hipKernelNodeParams kp{};
        if (hipGraphNodeGetType(nodes[i], &ty) != hipSuccess || ty != hipGraphNodeTypeKernel) continue;
        if (hipGraphKernelNodeGetParams(nodes[i], &kp) != hipSuccess) continue;
        if (kp.func == reinterpret_cast<void*>(&plan_mark_direct_kernel)) {
          p->mark_node = nodes[i];
          p->mark_params = kp;
        }
      }
    }
    if (!p->mark_node) rc = DAL_ERR_HIP;
  }
  if (cs) (void)hipStreamDestroy(cs);
  if (rc) {
    dal_dw_plan_destroy(p);
    return rc;
  }
  p->base_flags = base_flags;
  p->flags = flags;
  p->n = n;
  p->row_base = idx_base;
  p->k = k;
  p->out_pair = out_pair;
  p->dev_status = dev_status;
  *plan_out = p;
  return DAL_OK;
}

extern "C" int dal_dw_plan_run(dal_dw_plan_t* p, const int64_t* unl, int64_t n_unl, int64_t* out_idx,
                               double* out_scores, int32_t* status_out, dal_stream_t stream) {
  if (!p || !status_out || (!unl && n_unl)) return DAL_ERR_ARG;
  hipStream_t st = as_stream(stream);
  const DeviceGuard guard(st);
  if (!guard.ok() || guard.device() != p->device) return DAL_ERR_ARG;  // a stream of another device
  volatile PlanSlot* slot = p->slot;
  const uint32_t step = stamp_step(++p->step);
  // the 8-bit stamps wrapped: clear them (once per 255 replays) before this step marks its rows
  if (step == 1u && p->step > 1u && hipMemsetAsync(p->stamp, 0, static_cast<size_t>(p->n), st) != hipSuccess)
    return DAL_ERR_HIP;
  {
    hipKernelNodeParams np = p->mark_params;
    int64_t row_base = p->row_base, n = p->n;
    uint8_t* stamp = p->stamp;
    uint32_t* step_dev = p->step_dev;
    void* kargs[7] = {&unl, &n_unl, const_cast<uint32_t*>(&step), &row_base, &n, &stamp, &step_dev};
    np.kernelParams = kargs;
    np.extra = nullptr;
    if (hipGraphExecKernelNodeSetParams(p->exec, p->mark_node, &np) != hipSuccess) return DAL_ERR_HIP;
  }
  slot->out[0] = out_idx;
  slot->out[1] = reinterpret_cast<int64_t*>(out_scores);
  slot->status = -1;  // overwritten by the graph's last kernel
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (hipGraphLaunch(p->exec, st) != hipSuccess) return DAL_ERR_HIP;
  // the graph's last kernel publishes the status word last: spin on it (a
  // blocking stream sync wakes up tens of microseconds late), bounded, then
  // fall back to the sync.  Later work on the stream is ordered after the
  // graph anyway.
  const auto spin_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(20);
  while (slot->status < 0 && std::chrono::steady_clock::now() < spin_end) __builtin_ia32_pause();
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (slot->status < 0 && hipStreamSynchronize(st) != hipSuccess) return DAL_ERR_HIP;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  const int32_t v = slot->status;
  if (v < 0) return DAL_ERR_HIP;  // the step did not publish its status
  *status_out = v;
  return DAL_OK;
}

extern "C" int dal_dw_plan_launch(dal_dw_plan_t* p, const int64_t* unl, int64_t n_unl, dal_stream_t stream) {
  if (!p || (!unl && n_unl)) return DAL_ERR_ARG;
  hipStream_t st = as_stream(stream);
  const DeviceGuard guard(st);
  if (!guard.ok() || guard.device() != p->device) return DAL_ERR_ARG;
  const uint32_t step = stamp_step(++p->step);
  if (step == 1u && p->step > 1u && hipMemsetAsync(p->stamp, 0, static_cast<size_t>(p->n), st) != hipSuccess)
    return DAL_ERR_HIP;  // (as dal_dw_plan_run)
  hipKernelNodeParams np = p->mark_params;
  int64_t row_base = p->row_base, n = p->n;
  uint8_t* stamp = p->stamp;
  uint32_t* step_dev = p->step_dev;
  void* kargs[7] = {&unl, &n_unl, const_cast<uint32_t*>(&step), &row_base, &n, &stamp, &step_dev};
  np.kernelParams = kargs;
  np.extra = nullptr;
  if (hipGraphExecKernelNodeSetParams(p->exec, p->mark_node, &np) != hipSuccess) return DAL_ERR_HIP;
  volatile PlanSlot* slot = p->slot;
  slot->out[0] = nullptr;  // no publishing: the outputs stay in the plan's static buffers
  slot->out[1] = nullptr;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (hipGraphLaunch(p->exec, st) != hipSuccess) return DAL_ERR_HIP;
  return DAL_OK;
}

extern "C" void dal_dw_plan_destroy(dal_dw_plan_t* p) {
  if (!p) return;
  if (p->exec) (void)hipGraphExecDestroy(p->exec);
  if (p->graph) (void)hipGraphDestroy(p->graph);
  if (p->slot) (void)hipHostFree(p->slot);
  if (p->stamp) (void)hipFree(p->stamp);
  delete p;
}
