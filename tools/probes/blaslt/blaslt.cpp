// hipBLASLt GEMM node: plan building and launch (see blaslt.h).
#include "blaslt.h"

#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <stdexcept>
#include <string>

namespace kdl {

namespace {

constexpr int kMaxAlgos = 16;
constexpr uint64_t kMaxWorkspace = 64ull << 20;   // split-K algorithms; plenty of HBM

void ck(hipblasStatus_t s, const char* what) {
  if (s != HIPBLAS_STATUS_SUCCESS) throw std::runtime_error(std::string("hipBLASLt ") + what + " failed (" + std::to_string((int)s) + ")");
}

// one handle per device, created on first use and kept for the process lifetime
hipblasLtHandle_t handle_for_current_device() {
  static std::mutex mu;
  static std::map<int, hipblasLtHandle_t> handles;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) throw std::runtime_error("hipGetDevice failed");
  std::lock_guard<std::mutex> lk(mu);
  auto it = handles.find(dev);
  if (it != handles.end()) return it->second;
  hipblasLtHandle_t h = nullptr;
  ck(hipblasLtCreate(&h), "create");
  handles[dev] = h;
  return h;
}

}  // namespace

struct BlasLtPlan {
  hipblasLtHandle_t h = nullptr;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  int nalgos = 0;
  float alpha = 1.f, beta = 0.f;
  void* ws = nullptr;
  size_t ws_bytes = 0;

  ~BlasLtPlan() {
    if (ws) (void)hipFree(ws);
    if (la) hipblasLtMatrixLayoutDestroy(la);
    if (lb) hipblasLtMatrixLayoutDestroy(lb);
    if (lc) hipblasLtMatrixLayoutDestroy(lc);
    if (ld) hipblasLtMatrixLayoutDestroy(ld);
    if (desc) hipblasLtMatmulDescDestroy(desc);
  }
};

int blaslt_prepare(BlasLtArgs& a) {
  if (a.M <= 0 || a.N <= 0 || a.K <= 0 || !a.x || !a.w || !a.y || a.ldx < a.K || a.ldy < a.N ||
      (a.res && a.ldr < a.N))
    throw std::invalid_argument("blaslt: bad shape / pointers");
  auto p = std::make_shared<BlasLtPlan>();
  p->h = handle_for_current_device();
  if (a.dt == 2 && !a.wscale) throw std::invalid_argument("blaslt: e4m3 operands need the weight scales");
  const hipDataType et = a.dt == 1 ? HIP_R_16F : HIP_R_16BF;         // y / res
  const hipDataType it = a.dt == 2 ? HIP_R_8F_E4M3 : et;              // x / w
  ck(hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F), "desc");
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  ck(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)), "transA");
  ck(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)), "transB");
  if (a.act < 0 || a.act > 2) throw std::invalid_argument("blaslt: act is 0 (none), 1 (ReLU) or 2 (GELU)");
  static const hipblasLtEpilogue_t kEpi[2][3] = {
      {HIPBLASLT_EPILOGUE_DEFAULT, HIPBLASLT_EPILOGUE_RELU, HIPBLASLT_EPILOGUE_GELU},
      {HIPBLASLT_EPILOGUE_BIAS, HIPBLASLT_EPILOGUE_RELU_BIAS, HIPBLASLT_EPILOGUE_GELU_BIAS}};
  hipblasLtEpilogue_t epi = kEpi[a.bias ? 1 : 0][a.act];
  ck(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)), "epilogue");
  if (a.bias) {
    const void* bp = a.bias;
    const hipDataType bt = HIP_R_32F;
    ck(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)), "bias");
    ck(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)), "bias type");
  }
  if (a.dt == 2) {
    // D = wscale[n] * (W8 X8^T)[n][m] + bias + C: A (the weight, m = N rows) scaled per row
    const hipblasLtMatmulMatrixScale_t mode = HIPBLASLT_MATMUL_MATRIX_SCALE_OUTER_VEC_32F;
    const void* sp = a.wscale;
    ck(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_A_SCALE_MODE, &mode, sizeof(mode)), "scale mode");
    ck(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_A_SCALE_POINTER, &sp, sizeof(sp)), "scale A");
  }
  ck(hipblasLtMatrixLayoutCreate(&p->la, it, a.K, a.N, a.K), "layout A");
  ck(hipblasLtMatrixLayoutCreate(&p->lb, it, a.K, a.M, a.ldx), "layout B");
  ck(hipblasLtMatrixLayoutCreate(&p->lc, et, a.N, a.M, a.res ? a.ldr : a.ldy), "layout C");
  ck(hipblasLtMatrixLayoutCreate(&p->ld, et, a.N, a.M, a.ldy), "layout D");
  p->beta = a.res ? 1.f : 0.f;

  hipblasLtMatmulPreference_t pref = nullptr;
  ck(hipblasLtMatmulPreferenceCreate(&pref), "preference");
  const uint64_t wsmax = kMaxWorkspace;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsmax, sizeof(wsmax));
  hipblasLtMatmulHeuristicResult_t res[kMaxAlgos];
  int n = 0;
  const hipblasStatus_t hs =
      hipblasLtMatmulAlgoGetHeuristic(p->h, p->desc, p->la, p->lb, p->lc, p->ld, pref, kMaxAlgos, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  ck(hs, "heuristic");
  if (n <= 0) throw std::runtime_error("blaslt: no algorithm for this problem");
  const int pick = a.algo < 0 ? 0 : (a.algo >= n ? n - 1 : a.algo);
  p->algo = res[pick].algo;
  p->nalgos = n;
  p->ws_bytes = res[pick].workspaceSize;
  if (p->ws_bytes && hipMalloc(&p->ws, p->ws_bytes) != hipSuccess) throw std::runtime_error("blaslt: workspace alloc");
  a.plan = p;
  return n;
}

hipError_t blaslt_run(const BlasLtArgs& a, hipStream_t s) {
  const BlasLtPlan* p = a.plan.get();
  if (!p) return hipErrorNotReady;
  const void* c = a.res ? a.res : a.y;
  const hipblasStatus_t st = hipblasLtMatmul(p->h, p->desc, &p->alpha, a.w, p->la, a.x, p->lb, &p->beta, c, p->lc,
                                             a.y, p->ld, &p->algo, p->ws, p->ws_bytes, s);
  return st == HIPBLAS_STATUS_SUCCESS ? hipSuccess : hipErrorLaunchFailure;
}

hipError_t blaslt_run(BlasLtArgs& a, hipStream_t s) {
  if (!a.plan) blaslt_prepare(a);
  return blaslt_run(static_cast<const BlasLtArgs&>(a), s);
}

}  // namespace kdl
