// rphedge native runtime: hipGraph capture/replay, RCCL communicator over
// xGMI, layout self-check and small device helpers.  Exposed as a C ABI and
// bound from Python with ctypes (rphedge/ops/native.py) — no torch C++ ABI
// dependency, so the library loads into the torch process and shares its HIP
// runtime (same SONAME libamdhip64.so.7) and RCCL (librccl.so.1).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include "rph_types.h"

using namespace rph;

static thread_local char g_err[512];

static int set_err(const char* what, int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s failed (%d): %s", what, code, msg ? msg : "");
  return code == 0 ? -1 : code;
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) return set_err(#expr, (int)_e, hipGetErrorString(_e));   \
  } while (0)

#define NCCL_TRY(expr)                                                             \
  do {                                                                             \
    ncclResult_t _r = (expr);                                                      \
    if (_r != ncclSuccess) return set_err(#expr, (int)_r, ncclGetErrorString(_r)); \
  } while (0)

extern "C" const char* rph_last_error() { return g_err; }

// descriptor validation failures from the kernel launchers (hedge_mlp.hip)
namespace rph {
int rph_report(const char* what, const char* msg) { return set_err(what, -22, msg); }
}  // namespace rph

// ---------------------------------------------------------------------------
// Layout self-check: the Python ctypes mirrors compare every offset.
// ---------------------------------------------------------------------------
#define OFF(T, f) (long long)offsetof(T, f)
extern "C" int rph_layout(long long* out, int cap) {
  long long v[] = {
      (long long)sizeof(NetWeights), (long long)sizeof(OptState), (long long)sizeof(FitState),
      OFF(NetWeights, cur), OFF(OptState, t), OFF(OptState, lr), OFF(OptState, nan_steps),
      OFF(FitState, best_loss), OFF(FitState, stopped), OFF(FitState, epoch), OFF(FitState, last_loss),
      OFF(FitState, restore_at_end), OFF(FitState, hist),
      // TrainDesc
      (long long)sizeof(TrainDesc), OFF(TrainDesc, price), OFF(TrainDesc, target), OFF(TrainDesc, wts),
      OFF(TrainDesc, lr_sched), OFF(TrainDesc, slab), OFF(TrainDesc, counter), OFF(TrainDesc, grad_out),
      OFF(TrainDesc, bond), OFF(TrainDesc, inv_batch), OFF(TrainDesc, loss), OFF(TrainDesc, seed),
      OFF(TrainDesc, num_wgs), OFF(TrainDesc, head), OFF(TrainDesc, acc), OFF(TrainDesc, deterministic), OFF(TrainDesc, stamps),
      OFF(TrainDesc, dp_world), OFF(TrainDesc, dp_mbox), OFF(TrainDesc, dp_flags), OFF(TrainDesc, dp_counter), OFF(TrainDesc, dp_error),
      OFF(TrainDesc, fit_init), OFF(TrainDesc, fmu), OFF(TrainDesc, fisd),
      // EvalDesc
      (long long)sizeof(EvalDesc), OFF(EvalDesc, price_t), OFF(EvalDesc, price_t1), OFF(EvalDesc, target),
      OFF(EvalDesc, wa), OFF(EvalDesc, g_base), OFF(EvalDesc, v_out), OFF(EvalDesc, hold_out),
      OFF(EvalDesc, resid_out), OFF(EvalDesc, pred1_out), OFF(EvalDesc, stats), OFF(EvalDesc, bond_t),
      OFF(EvalDesc, hold_c), OFF(EvalDesc, n_local), OFF(EvalDesc, head), OFF(EvalDesc, fmu), OFF(EvalDesc, fisd),
      OFF(EvalDesc, snap_a), OFF(EvalDesc, snap_b),
      // PnlDesc
      (long long)sizeof(PnlDesc), OFF(PnlDesc, feat_ts), OFF(PnlDesc, price), OFF(PnlDesc, price_ts),
      OFF(PnlDesc, snap), OFF(PnlDesc, bond), OFF(PnlDesc, pnl_out), OFF(PnlDesc, stats), OFF(PnlDesc, alpha),
      OFF(PnlDesc, has_b), OFF(PnlDesc, n_dates), OFF(PnlDesc, head),
      // LmDesc + LM state layout
      (long long)sizeof(LmDesc), OFF(LmDesc, slab_b), OFF(LmDesc, slab_g), OFF(LmDesc, num_wgs),
      OFF(LmDesc, passes), OFF(LmDesc, gram_blk), OFF(LmDesc, inv_ns), OFF(LmDesc, lam0), OFF(LmDesc, ridge), OFF(LmDesc, bias_index), OFF(LmDesc, weights_only), OFF(LmDesc, damping), OFF(LmDesc, stop_tol), OFF(LmDesc, gram_skip),
      OFF(LmDesc, inst), OFF(LmDesc, lam_carry), OFF(LmDesc, w0), OFF(LmDesc, renorm), OFF(LmDesc, ren_isd), OFF(LmDesc, out_n), OFF(LmDesc, gfeat), OFF(LmDesc, gprice), OFF(LmDesc, gram_side), OFF(LmDesc, q_delta), OFF(LmDesc, dp), OFF(LmDesc, dp_fused), OFF(LmDesc, gtarget), OFF(LmDesc, gram_base), (long long)sizeof(LmDesc), (long long)LMS_LFIN, (long long)LMS_FAILTOT, (long long)LM_SEL_W, (long long)LM_DP_PITCH,
      (long long)sizeof(LmDpDesc), OFF(LmDpDesc, counter), OFF(LmDpDesc, world), OFF(LmDpDesc, pitch),
      (long long)LM_NPMAX, (long long)LM_RED, (long long)LMS_BEST, (long long)LMS_FLOATS,
      (long long)LM_SPEC, (long long)LMS_SPEC_W, (long long)LMS_SLOTS, (long long)LM_SLOT, (long long)LSS_LBEST, (long long)LSS_STOP,
      // SimDesc
      (long long)sizeof(SimDesc), OFF(SimDesc, path_offset), OFF(SimDesc, sv1), OFF(SimDesc, dims1),
      OFF(SimDesc, sv2), OFF(SimDesc, dims2), OFF(SimDesc, s0), OFF(SimDesc, chol), OFF(SimDesc, dt),
      OFF(SimDesc, inv_norm), OFF(SimDesc, v0), OFF(SimDesc, rho), OFF(SimDesc, l0), OFF(SimDesc, n0),
      OFF(SimDesc, seed), OFF(SimDesc, out), OFF(SimDesc, final2_out), OFF(SimDesc, sv_tscale),
      OFF(SimDesc, scheme), OFF(SimDesc, map_blk), OFF(SimDesc, map_stride),
      (long long)LAG_SLOTS,
  };
  const int n = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n && i < cap; ++i) out[i] = v[i];
  return n;
}

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------
extern "C" int rph_device_info(int dev, int* cus, int* lds_per_cu, long long* hbm_bytes, char* name, int name_cap) {
  hipDeviceProp_t p;
  HIP_TRY(hipGetDeviceProperties(&p, dev));
  *cus = p.multiProcessorCount;
  *lds_per_cu = (int)p.maxSharedMemoryPerMultiProcessor;
  *hbm_bytes = (long long)p.totalGlobalMem;
  snprintf(name, name_cap, "%s", p.gcnArchName);
  return 0;
}

extern "C" int rph_memset_async(void* ptr, int value, long long bytes, void* stream) {
  HIP_TRY(hipMemsetAsync(ptr, value, (size_t)bytes, (hipStream_t)stream));
  return 0;
}

extern "C" int rph_stream_sync(void* stream) {
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

// ---------------------------------------------------------------------------
// hipGraph capture / replay of whole training scans.
// ---------------------------------------------------------------------------
extern "C" int rph_graph_begin(void* stream) {
  HIP_TRY(hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeThreadLocal));
  return 0;
}

extern "C" int rph_graph_end(void* stream, void** exec_out, long long* num_nodes) {
  hipGraph_t g = nullptr;
  HIP_TRY(hipStreamEndCapture((hipStream_t)stream, &g));
  size_t nn = 0;
  HIP_TRY(hipGraphGetNodes(g, nullptr, &nn));
  *num_nodes = (long long)nn;
  hipGraphExec_t ex = nullptr;
  HIP_TRY(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  HIP_TRY(hipGraphDestroy(g));
  *exec_out = (void*)ex;
  return 0;
}

extern "C" int rph_graph_launch(void* exec, void* stream) {
  HIP_TRY(hipGraphLaunch((hipGraphExec_t)exec, (hipStream_t)stream));
  return 0;
}

extern "C" int rph_graph_destroy(void* exec) {
  HIP_TRY(hipGraphExecDestroy((hipGraphExec_t)exec));
  return 0;
}

// ---------------------------------------------------------------------------
// RCCL communicator (one per process/GPU).  The 128-byte unique id is
// generated on rank 0 and broadcast through the torch.distributed store by the
// Python side.  All-reduces are enqueued on the caller's (compute) stream so
// they can be captured into the same hipGraph as the training steps.
// ---------------------------------------------------------------------------
extern "C" int rph_nccl_unique_id(char* out128) {
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  memcpy(out128, &id, sizeof(id));
  return (int)sizeof(id);
}

extern "C" int rph_nccl_init(const char* id128, int nranks, int rank, void** comm_out) {
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  ncclComm_t c = nullptr;
  NCCL_TRY(ncclCommInitRank(&c, nranks, id, rank));
  *comm_out = (void*)c;
  return 0;
}

extern "C" int rph_nccl_allreduce_f32(void* comm, void* buf, long long count, void* stream) {
  NCCL_TRY(ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, ncclSum, (ncclComm_t)comm, (hipStream_t)stream));
  return 0;
}

extern "C" int rph_nccl_allreduce_f64(void* comm, void* buf, long long count, void* stream) {
  NCCL_TRY(ncclAllReduce(buf, buf, (size_t)count, ncclFloat64, ncclSum, (ncclComm_t)comm, (hipStream_t)stream));
  return 0;
}

extern "C" int rph_nccl_allreduce_u32(void* comm, void* buf, long long count, void* stream) {
  NCCL_TRY(ncclAllReduce(buf, buf, (size_t)count, ncclUint32, ncclSum, (ncclComm_t)comm, (hipStream_t)stream));
  return 0;
}

extern "C" int rph_nccl_destroy(void* comm) {
  NCCL_TRY(ncclCommDestroy((ncclComm_t)comm));
  return 0;
}

// ---------------------------------------------------------------------------
// IPC mailboxes for the fused xGMI all-reduce (one allocation per rank,
// exported with hipIpcGetMemHandle and opened by every peer process).
// ---------------------------------------------------------------------------
// Mailboxes are written by PEER GPUs over xGMI and polled locally, so they are
// allocated fine-grained (coherent across devices by memory type) when the
// driver can export such an allocation; otherwise coarse-grained hipMalloc
// (the kernels use system-scope stores/loads either way).
static int g_ipc_finegrained = -1;  // 1/0 once decided

extern "C" int rph_ipc_alloc(long long bytes, void** ptr_out, char* handle_out /*64 B*/) {
  void* p = nullptr;
  hipIpcMemHandle_t h;
  bool done = false;
  if (g_ipc_finegrained != 0 && hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocFinegrained) == hipSuccess) {
    if (hipIpcGetMemHandle(&h, p) == hipSuccess) {
      done = true;
      g_ipc_finegrained = 1;
    } else {
      (void)hipGetLastError();
      (void)hipFree(p);
      p = nullptr;
      g_ipc_finegrained = 0;
    }
  } else {
    (void)hipGetLastError();
  }
  if (!done) {
    HIP_TRY(hipMalloc(&p, (size_t)bytes));
    HIP_TRY(hipIpcGetMemHandle(&h, p));
  }
  HIP_TRY(hipMemset(p, 0, (size_t)bytes));
  HIP_TRY(hipDeviceSynchronize());
  memcpy(handle_out, &h, sizeof(h));
  *ptr_out = p;
  return 0;
}

extern "C" int rph_ipc_is_finegrained() { return g_ipc_finegrained; }

extern "C" int rph_ipc_open(const char* handle /*64 B*/, void** ptr_out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  HIP_TRY(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  *ptr_out = p;
  return 0;
}

extern "C" int rph_ipc_close(void* p) {
  HIP_TRY(hipIpcCloseMemHandle(p));
  return 0;
}

extern "C" int rph_free(void* p) {
  HIP_TRY(hipFree(p));
  return 0;
}

extern "C" int rph_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }
