// pybind11 bindings of the HIP kernel library + native executor (module kdl._C).
// Device pointers and hipStream_t travel as Python ints (torch: .data_ptr(),
// torch.cuda.current_stream().cuda_stream); no torch headers are needed, which
// keeps the extension a plain hipcc build (no hipify, no CUDA shims).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "kernels/launch.h"
#include "runtime/engine.h"
#include "runtime/comm.h"
#include "runtime/dp_hiploop.h"
#include "runtime/hip_backend.h"

namespace py = pybind11;
using namespace kdl;

namespace {

template <typename T>
T* P(const py::dict& d, const char* k) {
  if (!d.contains(k) || d[k].is_none()) return nullptr;
  return reinterpret_cast<T*>(d[k].cast<uintptr_t>());
}
int I(const py::dict& d, const char* k, int def = 0) {
  if (!d.contains(k) || d[k].is_none()) return def;
  return d[k].cast<int>();
}
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

ConvGemmArgs conv_args(const py::dict& d) {
  ConvGemmArgs a{};
  a.x = P<const uint16_t>(d, "x");
  a.wp = P<const uint16_t>(d, "wp");
  a.bias = P<const float>(d, "bias");
  a.dww = P<const float>(d, "dww");
  a.dwk = P<const uint16_t>(d, "dwk");
  a.res = P<const uint16_t>(d, "res");
  a.y = P<uint16_t>(d, "y");
  a.stamps = P<unsigned long long>(d, "stamps");
  a.B = I(d, "B"); a.H = I(d, "H"); a.W = I(d, "W");
  a.OH = I(d, "OH"); a.OW = I(d, "OW"); a.M = I(d, "M");
  a.ldx = I(d, "ldx"); a.ldy = I(d, "ldy"); a.ldr = I(d, "ldr");
  a.K = I(d, "K"); a.cin = I(d, "cin", 32); a.NF = I(d, "NF");
  a.nstore = I(d, "nstore"); a.stride = I(d, "stride", 1);
  a.relu_in = I(d, "relu_in"); a.relu_out = I(d, "relu_out"); a.opad = I(d, "opad");
  a.dt = I(d, "dt");
  a.krot = I(d, "krot");
  a.ksplit = I(d, "ksplit");
  a.ws = P<float>(d, "ws");
  a.cnt = P<int>(d, "cnt");
  a.ascale = P<const float>(d, "ascale");
  a.ascale_ld = I(d, "ascale_ld");
  return a;
}
float F(const py::dict& d, const char* k, float def) {
  if (!d.contains(k) || d[k].is_none()) return def;
  return d[k].cast<float>();
}
StemArgs stem_args(const py::dict& d) {
  StemArgs a{};
  a.x = P<const void>(d, "x"); a.wp = P<const uint16_t>(d, "wp");
  a.bias = P<const float>(d, "bias"); a.y = P<uint16_t>(d, "y");
  a.B = I(d, "B"); a.H = I(d, "H"); a.W = I(d, "W");
  a.OH = I(d, "OH"); a.OW = I(d, "OW"); a.ldy = I(d, "ldy"); a.in_kind = I(d, "in_kind");
  // defaults = the Xception stem (3x3 s2 'valid' -> 32, normalisation folded into the weights)
  a.KH = I(d, "KH", 3); a.KW = I(d, "KW", 3); a.stride = I(d, "stride", 2); a.pad = I(d, "pad", 0);
  a.cout = I(d, "cout", 32); a.relu = I(d, "relu", 1); a.dt = I(d, "dt");
  const char* sk[3] = {"scale0", "scale1", "scale2"};
  const char* hk[3] = {"shift0", "shift1", "shift2"};
  for (int c = 0; c < 3; ++c) { a.scale[c] = F(d, sk[c], 1.f); a.shift[c] = F(d, hk[c], 0.f); }
  a.rows = I(d, "rows", 0);
  return a;
}
GapArgs gap_args(const py::dict& d) {
  GapArgs a{};
  a.x = P<const uint16_t>(d, "x"); a.y = P<float>(d, "y"); a.yb = P<uint16_t>(d, "yb");
  a.B = I(d, "B"); a.HW = I(d, "HW"); a.ldx = I(d, "ldx"); a.F = I(d, "F"); a.dt = I(d, "dt");
  return a;
}
FcArgs fc_args(const py::dict& d) {
  FcArgs a{};
  a.x = P<const float>(d, "x"); a.w = P<const float>(d, "w"); a.bias = P<const float>(d, "bias");
  a.out = P<float>(d, "out");
  a.B = I(d, "B"); a.F = I(d, "F"); a.N = I(d, "N"); a.relu = I(d, "relu");
  return a;
}
PatchifyArgs patch_args(const py::dict& d) {
  PatchifyArgs a{};
  a.x = P<const uint8_t>(d, "x"); a.y = P<uint16_t>(d, "y");
  a.B = I(d, "B"); a.H = I(d, "H"); a.W = I(d, "W"); a.P = I(d, "P"); a.ldy = I(d, "ldy");
  const char* sk[3] = {"scale0", "scale1", "scale2"};
  const char* hk[3] = {"shift0", "shift1", "shift2"};
  for (int c = 0; c < 3; ++c) { a.scale[c] = F(d, sk[c], 1.f); a.shift[c] = F(d, hk[c], 0.f); }
  return a;
}
EmbedArgs embed_args(const py::dict& d) {
  EmbedArgs a{};
  a.x = P<uint16_t>(d, "x"); a.cls = P<const float>(d, "cls"); a.pos = P<const float>(d, "pos");
  a.B = I(d, "B"); a.T = I(d, "T"); a.D = I(d, "D");
  return a;
}
LnArgs ln_args(const py::dict& d) {
  LnArgs a{};
  a.x = P<const uint16_t>(d, "x"); a.y = P<uint16_t>(d, "y");
  a.gamma = P<const float>(d, "gamma"); a.beta = P<const float>(d, "beta");
  a.y8 = P<uint8_t>(d, "y8"); a.inv_scale = F(d, "inv_scale", 1.f);
  a.rows = d["rows"].cast<long>(); a.D = I(d, "D"); a.ldx = I(d, "ldx"); a.ldy = I(d, "ldy");
  a.eps = F(d, "eps", 1e-6f);
  return a;
}
AttnArgs attn_args(const py::dict& d) {
  AttnArgs a{};
  a.qkv = P<const uint16_t>(d, "qkv"); a.out = P<uint16_t>(d, "out");
  a.out8 = P<uint8_t>(d, "out8"); a.inv_scale = F(d, "inv_scale", 1.f);
  a.B = I(d, "B"); a.T = I(d, "T"); a.H = I(d, "H"); a.dh = I(d, "dh", 64);
  a.scale = F(d, "scale", 0.125f);
  return a;
}
DwkArgs dwk_args(const py::dict& d) {
  DwkArgs a{};
  a.x = P<const uint16_t>(d, "x"); a.w = P<const float>(d, "w"); a.bias = P<const float>(d, "bias");
  a.y = P<uint16_t>(d, "y"); a.pool = P<float>(d, "pool"); a.w1 = P<const float>(d, "w1");
  a.B = I(d, "B"); a.H = I(d, "H"); a.W = I(d, "W"); a.C = I(d, "C"); a.OH = I(d, "OH"); a.OW = I(d, "OW");
  a.K = I(d, "K"); a.S = I(d, "S", 1); a.pad = I(d, "pad"); a.act = I(d, "act"); a.Cs = I(d, "Cs");
  a.cg = I(d, "cg", 0); a.rb = I(d, "rb", 0); a.tw = I(d, "tw", 0); a.seg = I(d, "seg", 0);
  a.lds_kb = I(d, "lds_kb", 0); a.algo = I(d, "algo", 0); a.pd = I(d, "pd", 0);
  return a;
}
SeArgs se_args(const py::dict& d) {
  SeArgs a{};
  a.pool = P<const float>(d, "pool"); a.b1 = P<const float>(d, "b1");
  a.w2t = P<const float>(d, "w2t"); a.b2 = P<const float>(d, "b2"); a.scale = P<float>(d, "scale");
  a.B = I(d, "B"); a.ntiles = I(d, "ntiles"); a.HW = I(d, "HW"); a.C = I(d, "C"); a.Cs = I(d, "Cs");
  return a;
}
ChScaleArgs chs_args(const py::dict& d) {
  ChScaleArgs a{};
  a.y = P<uint16_t>(d, "y"); a.scale = P<const float>(d, "scale");
  a.B = I(d, "B"); a.HW = I(d, "HW"); a.C = I(d, "C");
  return a;
}
GemmF8Args f8_args(const py::dict& d) {
  GemmF8Args a{};
  a.x = P<const uint8_t>(d, "x"); a.wp = P<const uint8_t>(d, "wp"); a.bias = P<const float>(d, "bias");
  a.colscale = P<const float>(d, "colscale"); a.res = P<const uint16_t>(d, "res");
  a.y = P<uint16_t>(d, "y"); a.y8 = P<uint8_t>(d, "y8"); a.out_inv_scale = F(d, "out_inv_scale", 1.f);
  a.M = I(d, "M"); a.K = I(d, "K"); a.ldx = I(d, "ldx"); a.ldy = I(d, "ldy"); a.ldr = I(d, "ldr");
  a.NF = I(d, "NF"); a.nstore = I(d, "nstore"); a.relu_out = I(d, "relu_out");
  a.krot = I(d, "krot");
  return a;
}
EntryBlockArgs eb_args(const py::dict& d) {
  EntryBlockArgs a{};
  a.x = P<const uint16_t>(d, "x"); a.y = P<uint16_t>(d, "y");
  a.w1 = P<const uint16_t>(d, "w1"); a.b1 = P<const float>(d, "b1"); a.dw1 = P<const float>(d, "dw1");
  a.w2 = P<const uint16_t>(d, "w2"); a.b2 = P<const float>(d, "b2"); a.dw2 = P<const float>(d, "dw2");
  a.dwk1 = P<const uint16_t>(d, "dwk1"); a.dwk2 = P<const uint16_t>(d, "dwk2");
  a.wr = P<const uint16_t>(d, "wr"); a.br = P<const float>(d, "br");
  a.B = I(d, "B"); a.H = I(d, "H"); a.W = I(d, "W"); a.OH = I(d, "OH"); a.OW = I(d, "OW");
  a.ldx = I(d, "ldx"); a.ldy = I(d, "ldy"); a.grid = I(d, "grid");
  a.steps = P<const int4>(d, "steps"); a.step_off = P<const int>(d, "step_off");
  a.stamps = P<unsigned long long>(d, "stamps");
  if (!a.x || !a.y || !a.w1 || !a.b1 || !a.dw1 || !a.w2 || !a.b2 || !a.dw2 || !a.wr || !a.br)
    throw std::invalid_argument("entry_block: null pointer");
  return a;
}

FcMfmaArgs fcm_args(const py::dict& d) {
  FcMfmaArgs a{};
  a.xb = P<const uint16_t>(d, "xb"); a.wp = P<const uint16_t>(d, "wp"); a.bias = P<const float>(d, "bias");
  a.out = P<float>(d, "out");
  a.B = I(d, "B"); a.F = I(d, "F"); a.N = I(d, "N"); a.NF = I(d, "NF"); a.relu = I(d, "relu");
  a.dt = I(d, "dt");
  return a;
}
PoolAddArgs pool_args(const py::dict& d) {
  PoolAddArgs a{};
  a.x = P<const uint16_t>(d, "x"); a.res = P<const uint16_t>(d, "res"); a.y = P<uint16_t>(d, "y");
  a.B = I(d, "B"); a.H = I(d, "H"); a.W = I(d, "W"); a.OH = I(d, "OH"); a.OW = I(d, "OW");
  a.C = I(d, "C"); a.pad_top = I(d, "pad_top"); a.pad_left = I(d, "pad_left"); a.dt = I(d, "dt");
  a.algo = d.contains("algo") ? I(d, "algo") : 0;
  a.seg = d.contains("seg") ? I(d, "seg") : 0; a.rb = d.contains("rb") ? I(d, "rb") : 0;
  return a;
}
HeadArgs head_args(const py::dict& d) {
  HeadArgs a{};
  a.x = P<const uint16_t>(d, "x"); a.w1 = P<const float>(d, "w1"); a.b1 = P<const float>(d, "b1");
  a.w2 = P<const float>(d, "w2"); a.b2 = P<const float>(d, "b2"); a.out = P<float>(d, "out");
  a.feat = P<float>(d, "feat"); a.hid = P<float>(d, "hid");
  a.B = I(d, "B"); a.HW = I(d, "HW"); a.ldx = I(d, "ldx"); a.F = I(d, "F"); a.H1 = I(d, "H1");
  a.NC = I(d, "NC");
  return a;
}
ResizeArgs resize_args(const py::dict& d) {
  ResizeArgs a{};
  a.src = P<const uint8_t>(d, "src"); a.dst = P<uint8_t>(d, "dst");
  a.ytab = P<const int>(d, "ytab"); a.xtab = P<const int>(d, "xtab");
  a.SH = I(d, "SH"); a.SW = I(d, "SW"); a.OH = I(d, "OH"); a.OW = I(d, "OW"); a.n = I(d, "n", 1);
  return a;
}

DwArgs dw_args(const py::dict& d) {
  DwArgs a{};
  a.x = P<const uint16_t>(d, "x"); a.w = P<const float>(d, "w"); a.y = P<uint16_t>(d, "y");
  a.B = I(d, "B"); a.H = I(d, "H"); a.W = I(d, "W"); a.C = I(d, "C"); a.relu_in = I(d, "relu_in");
  a.cg = d.contains("cg") ? I(d, "cg") : 0; a.rb = d.contains("rb") ? I(d, "rb") : 0;
  a.tw = d.contains("tw") ? I(d, "tw") : 0; a.seg = d.contains("seg") ? I(d, "seg") : 0;
  a.algo = d.contains("algo") ? I(d, "algo") : 0; a.pd = d.contains("pd") ? I(d, "pd") : 0;
  return a;
}

void chk(hipError_t e, const char* what) { check_hip(e, what); }

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "kdl MI355X (gfx950) HIP kernels and native executor";

  m.def("conv_gemm", [](int mode, int cfg, py::dict d, uintptr_t s) {
    const auto a = conv_args(d);
    py::gil_scoped_release nogil;
    chk(conv_gemm(mode, cfg, a, S(s)), "conv_gemm");
  });
  m.def("conv_gemm_config", [](int cfg) {
    int bm = 0, bn = 0, th = 0;
    if (conv_gemm_config(cfg, &bm, &bn, &th) != 0) throw std::out_of_range("bad conv_gemm config");
    return py::make_tuple(bm, bn, th);
  });
  m.def("conv_gemm_num_configs", &conv_gemm_num_configs);
  // raw async copy (kind: hipMemcpyKind, 1 = H2D, 2 = D2H): the pipelined ingress /
  // egress of bench.py and the serving executor without torch's per-copy bookkeeping
  m.def("memcpy_async", [](uintptr_t dst, uintptr_t src, size_t n, int kind, uintptr_t s) {
    py::gil_scoped_release nogil;
    chk(hipMemcpyAsync((void*)dst, (const void*)src, n, (hipMemcpyKind)kind, S(s)), "memcpy_async");
  });
  m.def("dw3x3", [](py::dict d, uintptr_t s) {
    const auto a = dw_args(d);
    py::gil_scoped_release nogil;
    chk(dw3x3(a, S(s)), "dw3x3");
  });
  m.def("stem_conv", [](py::dict d, uintptr_t s) {
    const auto a = stem_args(d);
    py::gil_scoped_release nogil;
    chk(stem_conv(a, S(s)), "stem_conv");
  });
  m.def("pool_add", [](py::dict d, uintptr_t s) {
    const auto a = pool_args(d);
    py::gil_scoped_release nogil;
    chk(pool_add(a, S(s)), "pool_add");
  });
  m.def("head_dense", [](py::dict d, uintptr_t s) {
    const auto a = head_args(d);
    py::gil_scoped_release nogil;
    chk(head_dense(a, S(s)), "head_dense");
  });
  m.def("gap", [](py::dict d, uintptr_t s) {
    const auto a = gap_args(d);
    py::gil_scoped_release nogil;
    chk(gap(a, S(s)), "gap");
  });
  m.def("fc", [](py::dict d, uintptr_t s) {
    const auto a = fc_args(d);
    py::gil_scoped_release nogil;
    chk(fc(a, S(s)), "fc");
  });
  m.def("patchify", [](py::dict d, uintptr_t s) {
    const auto a = patch_args(d);
    py::gil_scoped_release nogil;
    chk(patchify(a, S(s)), "patchify");
  });
  m.def("embed_tokens", [](py::dict d, uintptr_t s) {
    const auto a = embed_args(d);
    py::gil_scoped_release nogil;
    chk(embed_tokens(a, S(s)), "embed_tokens");
  });
  m.def("layernorm", [](py::dict d, uintptr_t s) {
    const auto a = ln_args(d);
    py::gil_scoped_release nogil;
    chk(layernorm(a, S(s)), "layernorm");
  });
  m.def("attention", [](py::dict d, uintptr_t s) {
    const auto a = attn_args(d);
    py::gil_scoped_release nogil;
    chk(attention(a, S(s)), "attention");
  });
  m.def("dwk", [](py::dict d, uintptr_t s) {
    const auto a = dwk_args(d);
    py::gil_scoped_release nogil;
    chk(dwk(a, S(s)), "dwk");
  });
  m.def("dwk_tiles", [](py::dict d) {
    const auto a = dwk_args(d);
    int cg, rb, tw, nt;
    dwk_tiles(a, &cg, &rb, &tw, &nt);
    return py::make_tuple(cg, rb, tw, nt, dwk_seg(a));
  });
  m.def("squeeze_excite", [](py::dict d, uintptr_t s) {
    const auto a = se_args(d);
    py::gil_scoped_release nogil;
    chk(squeeze_excite(a, S(s)), "squeeze_excite");
  });
  m.def("channel_scale", [](py::dict d, uintptr_t s) {
    const auto a = chs_args(d);
    py::gil_scoped_release nogil;
    chk(channel_scale(a, S(s)), "channel_scale");
  });
  m.def("entry_block", [](int cfg, py::dict d, uintptr_t s) {
    const auto a = eb_args(d);
    py::gil_scoped_release nogil;
    chk(entry_block(cfg, a, S(s)), "entry_block");
  });
  m.def("entry_block_config", [](int cfg) {
    int c0 = 0, c1 = 0, pc = 0, lds = 0, occ = 0;
    if (entry_block_config(cfg, &c0, &c1, &pc, &lds, &occ) != 0) throw std::out_of_range("bad entry_block config");
    return py::make_tuple(c0, c1, pc, lds, occ);
  });
  m.def("gemm_f8", [](int cfg, py::dict d, uintptr_t s) {
    const auto a = f8_args(d);
    py::gil_scoped_release nogil;
    chk(gemm_f8(cfg, a, S(s)), "gemm_f8");
  });
  m.def("gemm_f8_config", [](int cfg) {
    int bm = 0, bn = 0, th = 0;
    if (gemm_f8_config(cfg, &bm, &bn, &th) != 0) throw std::out_of_range("bad gemm_f8 config");
    return py::make_tuple(bm, bn, th);
  });
  m.def("fc_mfma", [](py::dict d, uintptr_t s) {
    const auto a = fcm_args(d);
    py::gil_scoped_release nogil;
    chk(fc_mfma(a, S(s)), "fc_mfma");
  });
  m.def("resize_nearest_u8", [](py::dict d, uintptr_t s) {
    const auto a = resize_args(d);
    py::gil_scoped_release nogil;
    chk(resize_nearest_u8(a, S(s)), "resize_nearest_u8");
  });
  m.def("u8_to_bf16_norm", [](uintptr_t x, uintptr_t y, long npix, int ldy, uintptr_t s) {
    py::gil_scoped_release nogil;
    chk(u8_to_bf16_norm(reinterpret_cast<const uint8_t*>(x), reinterpret_cast<uint16_t*>(y), npix, ldy, S(s)),
        "u8_to_bf16_norm");
  });

  // device backend of the native batch executor (kdl._rt.Executor drives it from a C++ thread)
  py::class_<HipExecBackend>(m, "HipExecBackend")
      .def(py::init([](int device, int nslots, size_t item_bytes, int max_batch, int out_cols, uintptr_t copy_stream,
                       bool timing) {
             return new HipExecBackend(device, nslots, item_bytes, max_batch, out_cols, S(copy_stream), timing);
           }),
           py::arg("device"), py::arg("nslots"), py::arg("item_bytes"), py::arg("max_batch"), py::arg("out_cols"),
           py::arg("copy_stream") = 0, py::arg("timing") = true)
      // progs[slot][parity][stage]: Program objects kept alive by the caller
      .def("add_recipe", [](HipExecBackend& be, int bucket, std::vector<uintptr_t> streams, std::vector<int> wait_for,
                            py::list progs, std::vector<uintptr_t> dev_in, std::vector<uintptr_t> dev_out) {
        std::vector<hipStream_t> st;
        for (auto v : streams) st.push_back(S(v));
        std::vector<std::vector<std::vector<const Program*>>> pp;
        for (auto slot : progs) {
          std::vector<std::vector<const Program*>> ps;
          for (auto par : slot.cast<py::list>()) {
            std::vector<const Program*> pk;
            for (auto prog : par.cast<py::list>()) pk.push_back(&prog.cast<const Program&>());
            ps.push_back(pk);
          }
          pp.push_back(ps);
        }
        std::vector<void*> di, dout;
        for (auto v : dev_in) di.push_back(reinterpret_cast<void*>(v));
        for (auto v : dev_out) dout.push_back(reinterpret_cast<void*>(v));
        be.add_recipe(bucket, st, wait_for, pp, di, dout);
      })
      .def("api_ptr", [](const HipExecBackend& be) { return reinterpret_cast<uintptr_t>(be.api()); })
      .def("staging_ptr", [](HipExecBackend& be, int slot) { return reinterpret_cast<uintptr_t>(be.staging(slot)); })
      // direct use without the executor (tests): issue + complete of one slot
      .def("run", [](HipExecBackend& be, int slot, int bucket, int n_real) {
        py::gil_scoped_release nogil;
        const float* out = nullptr;
        kdl_device_times t{};
        if (be.issue(slot, bucket, n_real) != 0 || be.complete(slot, &out, &t) != 0)
          throw std::runtime_error("HipExecBackend: batch failed");
        return std::make_tuple(reinterpret_cast<uintptr_t>(out), t.h2d_ms, t.forward_ms, t.d2h_ms);
      });

  // ---- RCCL data-parallel serving (runtime/comm.h)
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init([](py::bytes id, int nranks, int rank, int device) {
             const std::string s = id;
             py::gil_scoped_release nogil;       // every rank blocks here until all have joined
             return new RcclComm(s, nranks, rank, device);
           }),
           py::arg("id"), py::arg("nranks"), py::arg("rank"), py::arg("device"))
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def("abort", &RcclComm::abort)
      .def("async_error", &RcclComm::async_error)
      // gather `nbytes` per rank to rank 0 on `stream` (device pointers); no extra stream
      .def("gather", [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t nbytes, uintptr_t stream) {
        if (rccl_gather(c, reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), nbytes, S(stream)) != 0)
          throw std::runtime_error("rccl_gather failed");
      });
  py::class_<DpLeader>(m, "DpLeader")
      .def(py::init([](HipExecBackend* local, RcclComm* sc, RcclComm* ga, std::vector<int> buckets, double timeout_s,
                       double ping_s) { return new DpLeader(local, sc, ga, std::move(buckets), timeout_s, ping_s); }),
           py::arg("local"), py::arg("scatter"), py::arg("gather"), py::arg("rank_buckets"), py::arg("timeout_s") = 120.0,
           py::arg("ping_s") = 0.0, py::keep_alive<1, 2>(), py::keep_alive<1, 3>(), py::keep_alive<1, 4>())
      .def("api_ptr", [](const DpLeader& l) { return reinterpret_cast<uintptr_t>(l.api()); })
      .def_property_readonly("world", &DpLeader::world)
      .def_property_readonly("steps", &DpLeader::steps)
      .def_property_readonly("broken", &DpLeader::broken)
      .def("send_ctrl", [](DpLeader& l, int cmd, int version) {
        py::gil_scoped_release nogil;
        return l.send_ctrl(cmd, version);
      })
      .def("ping", [](DpLeader& l) {
        py::gil_scoped_release nogil;
        return l.ping();
      })
      // direct use without the executor (tests / bench): issue + complete of one slot
      .def("run", [](DpLeader& l, int slot, int bucket, int n_real) {
        py::gil_scoped_release nogil;
        const float* out = nullptr;
        kdl_device_times t{};
        if (l.issue(slot, bucket, n_real) != 0 || l.complete(slot, &out, &t) != 0)
          throw std::runtime_error("DpLeader: step failed");
        return reinterpret_cast<uintptr_t>(out);
      });
  py::class_<DpFollower>(m, "DpFollower")
      .def(py::init([](HipExecBackend* local, RcclComm* sc, RcclComm* ga) { return new DpFollower(local, sc, ga); }),
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>(), py::keep_alive<1, 4>())
      .def_property_readonly("steps", &DpFollower::steps)
      // serve until DP_STOP / DP_RELOAD; returns (cmd, version, seq). Raises RuntimeError when rank 0
      // is silent for liveness_s (it pings while idle) or a communicator failed.
      .def("run", [](DpFollower& f, double liveness_s) {
        DpCtrl c{};
        {
          py::gil_scoped_release nogil;
          c = f.run(liveness_s);
        }
        return std::make_tuple(c.cmd, c.version, c.seq);
      }, py::arg("liveness_s") = 30.0);
  // ---- the same protocol over the HIP loopback platform (runtime/dp_hiploop.h): real engines,
  // streams and events on one GPU, ranks as threads of this process, device-to-device transport
  m.def("hiploop_unique_id", []() { return loop::unique_id(); });
  // module_local: kdl._rt registers the same C++ type (loop::Comm) as LoopComm
  py::class_<loop::Comm>(m, "HipLoopComm", py::module_local())
      .def(py::init<const std::string&, int, int>(), py::arg("id"), py::arg("nranks"), py::arg("rank"))
      .def_property_readonly("rank", &loop::Comm::rank)
      .def_property_readonly("size", &loop::Comm::size)
      .def("kill", &loop::Comm::kill)           // this rank stops matching: a dead process
      .def("abort", &loop::Comm::abort)
      .def("error", &loop::Comm::error);
  struct HLLeader {
    std::unique_ptr<HipLoopLocal> local;
    std::unique_ptr<HipLoopDpLeader> lead;
  };
  struct HLFollower {
    std::unique_ptr<HipLoopLocal> local;
    std::unique_ptr<HipLoopDpFollower> f;
  };
  py::class_<HLLeader>(m, "HipLoopDpLeader")
      .def(py::init([](HipExecBackend* be, loop::Comm* sc, loop::Comm* ga, std::vector<int> buckets, double timeout_s,
                       double ping_s) {
             auto h = new HLLeader();
             h->local = std::make_unique<HipLoopLocal>(be);
             h->lead = std::make_unique<HipLoopDpLeader>(h->local.get(), sc, ga, std::move(buckets), timeout_s, ping_s);
             return h;
           }),
           py::arg("local"), py::arg("scatter"), py::arg("gather"), py::arg("rank_buckets"), py::arg("timeout_s") = 120.0,
           py::arg("ping_s") = 0.0, py::keep_alive<1, 2>(), py::keep_alive<1, 3>(), py::keep_alive<1, 4>())
      .def("api_ptr", [](const HLLeader& l) { return reinterpret_cast<uintptr_t>(l.lead->api()); })
      .def_property_readonly("world", [](const HLLeader& l) { return l.lead->world(); })
      .def_property_readonly("steps", [](const HLLeader& l) { return l.lead->steps(); })
      .def_property_readonly("broken", [](const HLLeader& l) { return l.lead->broken(); })
      .def("send_ctrl", [](HLLeader& l, int cmd, int version) {
        py::gil_scoped_release nogil;
        return l.lead->send_ctrl(cmd, version);
      })
      .def("ping", [](HLLeader& l) {
        py::gil_scoped_release nogil;
        return l.lead->ping();
      });
  py::class_<HLFollower>(m, "HipLoopDpFollower")
      .def(py::init([](HipExecBackend* be, loop::Comm* sc, loop::Comm* ga) {
             auto h = new HLFollower();
             h->local = std::make_unique<HipLoopLocal>(be);
             h->f = std::make_unique<HipLoopDpFollower>(h->local.get(), sc, ga);
             return h;
           }),
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>(), py::keep_alive<1, 4>())
      .def_property_readonly("steps", [](const HLFollower& f) { return f.f->steps(); })
      .def("run", [](HLFollower& f, double liveness_s) {
        DpCtrl c{};
        {
          py::gil_scoped_release nogil;
          c = f.f->run(liveness_s);
        }
        return std::make_tuple(c.cmd, c.version, c.seq);
      }, py::arg("liveness_s") = 30.0);
  m.attr("DP_STOP") = int(DP_STOP);
  m.attr("DP_BATCH") = int(DP_BATCH);
  m.attr("DP_RELOAD") = int(DP_RELOAD);
  m.attr("DP_PING") = int(DP_PING);

  py::class_<Program>(m, "Program")
      .def(py::init<>())
      .def("add_conv_gemm", [](Program& p, const std::string& name, int mode, int cfg, py::dict d) {
        Op op; op.kind = OP_CONV_GEMM; op.name = name; op.mode = mode; op.cfg = cfg; op.g = conv_args(d);
        p.add(op);
      })
      .def("add_stem", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_STEM; op.name = name; op.st = stem_args(d); p.add(op);
      })
      .def("add_pool_add", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_POOL_ADD; op.name = name; op.pa = pool_args(d); p.add(op);
      })
      .def("add_head", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_HEAD; op.name = name; op.hd = head_args(d); p.add(op);
      })
      .def("add_gap", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_GAP; op.name = name; op.gp = gap_args(d); p.add(op);
      })
      .def("add_fc", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_FC; op.name = name; op.fc = fc_args(d); p.add(op);
      })
      .def("add_patchify", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_PATCHIFY; op.name = name; op.pt = patch_args(d); p.add(op);
      })
      .def("add_embed", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_EMBED; op.name = name; op.em = embed_args(d); p.add(op);
      })
      .def("add_layernorm", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_LN; op.name = name; op.ln = ln_args(d); p.add(op);
      })
      .def("add_attention", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_ATTN; op.name = name; op.at = attn_args(d); p.add(op);
      })
      .def("add_dwk", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_DWK; op.name = name; op.dk = dwk_args(d); p.add(op);
      })
      .def("add_se", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_SE; op.name = name; op.se = se_args(d); p.add(op);
      })
      .def("add_chscale", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_CHSCALE; op.name = name; op.cs = chs_args(d); p.add(op);
      })
      .def("add_entry_block", [](Program& p, const std::string& name, int cfg, py::dict d) {
        Op op; op.kind = OP_ENTRY_BLOCK; op.name = name; op.cfg = cfg; op.eb = eb_args(d); p.add(op);
      })
      .def("add_gemm_f8", [](Program& p, const std::string& name, int cfg, py::dict d) {
        Op op; op.kind = OP_GEMM_F8; op.name = name; op.cfg = cfg; op.f8 = f8_args(d); p.add(op);
      })
      .def("add_fc_mfma", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_FC_MFMA; op.name = name; op.fcm = fcm_args(d); p.add(op);
      })
      .def("add_resize", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_RESIZE; op.name = name; op.rs = resize_args(d); p.add(op);
      })
      .def("add_dw", [](Program& p, const std::string& name, py::dict d) {
        Op op; op.kind = OP_DW; op.name = name; op.dw = dw_args(d); p.add(op);
      })
      .def("add_memset", [](Program& p, const std::string& name, uintptr_t ptr, size_t bytes) {
        Op op; op.kind = OP_MEMSET; op.name = name; op.mem_ptr = reinterpret_cast<void*>(ptr);
        op.mem_bytes = bytes; p.add(op);
      })
      .def("set_cfg", [](Program& p, size_t i, int cfg) { p.mutable_op(i).cfg = cfg; })
      .def("cfg", [](const Program& p, size_t i) { return p.op(i).cfg; })
      .def("op_names", [](const Program& p) {
        std::vector<std::string> v;
        for (size_t i = 0; i < p.size(); ++i) v.push_back(p.op(i).name);
        return v;
      })
      .def("__len__", &Program::size)
      .def("run", [](const Program& p, uintptr_t s) { py::gil_scoped_release nogil; p.run(S(s)); })
      .def("capture", [](Program& p, uintptr_t s) { py::gil_scoped_release nogil; p.capture(S(s)); })
      .def("launch", [](const Program& p, uintptr_t s) { py::gil_scoped_release nogil; p.launch(S(s)); })
      .def("reset", &Program::reset)
      .def_property_readonly("captured", &Program::captured)
      .def("profile", [](const Program& p, uintptr_t s, int iters) {
        py::gil_scoped_release nogil;
        return p.profile(S(s), iters);
      });
}
