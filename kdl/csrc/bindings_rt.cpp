// pybind11 bindings of the CPU-only native runtime (module kdl._rt): dynamic
// batcher, TF-Serving Predict wire codec, TensorBundle SSTable reader.
// Every blocking call releases the GIL so gRPC handler threads and the per-GPU
// executor threads run truly concurrently.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <fstream>
#include <sstream>

#include "runtime/batcher.h"
#include "runtime/dp_loop.h"
#include "runtime/dp_schedule.h"
#include "runtime/executor.h"
#include "runtime/grpc_front.h"
#include "runtime/grpc_load.h"
#include "runtime/h2.h"
#include "runtime/sstable.h"
#include "runtime/tfproto.h"

namespace py = pybind11;
using namespace kdl;

namespace {

py::dict spec_dict(const ModelSpecView& s) {
  py::dict d;
  d["name"] = s.name;
  d["signature_name"] = s.signature_name;
  d["version_label"] = s.version_label;
  d["version"] = s.version;
  return d;
}

// the GIL must be free while the front joins its threads (slow-path threads take it), and
// held while its Python slow-path callable is released
struct FrontDeleter {
  void operator()(GrpcFront* f) const {
    {
      py::gil_scoped_release nogil;
      f->stop();
    }
    delete f;
  }
};

}  // namespace

PYBIND11_MODULE(_rt, m) {
  m.doc() = "kdl native CPU runtime: dynamic batcher, TF-Serving wire codec, TensorBundle reader";
  m.def("now_us", &now_us);

  py::register_exception<ProtoError>(m, "ProtoError", PyExc_ValueError);

  // data-parallel message schedule (runtime/dp_schedule.h): the exact per-rank op lists the
  // RCCL backend posts, exposed so a CPU test can match every rank's sends against its peers'
  auto msgs_py = [](const std::vector<DpMsg>& v) {
    py::list out;
    for (const auto& m : v) out.append(py::make_tuple(m.channel, m.send, m.peer, m.bytes, m.what, m.group));
    return out;
  };
  m.def("dp_leader_step", [msgs_py](int world, size_t item_bytes, int out_cols, int cmd, int shard) {
    return msgs_py(dp_leader_step(DpGeometry{world, item_bytes, out_cols}, cmd, shard));
  });
  m.def("dp_follower_step", [msgs_py](int world, size_t item_bytes, int out_cols, int cmd, int shard, bool next) {
    return msgs_py(dp_follower_step(DpGeometry{world, item_bytes, out_cols}, cmd, shard, next));
  });
  m.def("dp_plan_shard", &dp_plan_shard);

  m.def("f32_to_u8_exact", [](py::buffer src, py::buffer dst) {
    py::buffer_info si = src.request(), di = dst.request(true);
    const size_t n = (size_t)si.size * si.itemsize / 4;
    if ((size_t)di.size * di.itemsize < n) throw std::invalid_argument("f32_to_u8_exact: dst too small");
    py::gil_scoped_release nogil;
    return f32_to_u8_exact(static_cast<const float*>(si.ptr), static_cast<uint8_t*>(di.ptr), n);
  });
  m.attr("DP_CTRL_BYTES") = int(sizeof(DpCtrl));

  m.def("parse_predict_request", [](py::bytes req) {
    std::string_view sv = req;  // zero-copy view of the Python bytes
    PredictRequestView v;
    {
      py::gil_scoped_release nogil;
      v = parse_predict_request(reinterpret_cast<const uint8_t*>(sv.data()), sv.size());
    }
    py::dict out;
    out["model_spec"] = spec_dict(v.spec);
    py::list inputs;
    for (auto& kv : v.inputs) {
      const TensorView& t = kv.second;
      py::dict td;
      td["key"] = kv.first;
      td["dtype"] = t.dtype;
      td["dims"] = t.dims;
      td["unknown_rank"] = t.unknown_rank;
      td["has_content"] = t.has_content;
      td["values_field"] = t.values_field;
      td["offset"] = t.content_offset;
      td["size"] = t.content_size;
      td["unpacked"] = py::bytes(reinterpret_cast<const char*>(t.unpacked.data()), t.unpacked.size());
      inputs.append(td);
    }
    out["inputs"] = inputs;
    out["output_filter"] = v.output_filter;
    return out;
  });
  m.def("parse_model_spec_request", [](py::bytes req) {
    std::string_view sv = req;
    return spec_dict(parse_model_spec_request(reinterpret_cast<const uint8_t*>(sv.data()), sv.size()));
  });
  m.def("build_predict_response",
        [](py::list outputs, const std::string& name, int64_t version, const std::string& signature) {
          std::vector<OutputTensor> outs;
          std::vector<py::array_t<float, py::array::c_style | py::array::forcecast>> keep;
          for (auto item : outputs) {
            auto tup = item.cast<py::tuple>();
            auto arr = tup[1].cast<py::array_t<float, py::array::c_style | py::array::forcecast>>();
            keep.push_back(arr);
            OutputTensor o;
            o.key = tup[0].cast<std::string>();
            for (py::ssize_t i = 0; i < arr.ndim(); ++i) o.dims.push_back(arr.shape(i));
            o.values = arr.data();
            outs.push_back(o);
          }
          ModelSpecView s;
          s.name = name;
          s.version = version;
          s.signature_name = signature;
          std::string b = build_predict_response(outs, s);
          return py::bytes(b);
        });

  m.def("crc32c", [](py::bytes b, uint32_t init) {
    std::string_view sv = b;
    return crc32c(reinterpret_cast<const uint8_t*>(sv.data()), sv.size(), init);
  }, py::arg("data"), py::arg("init") = 0);
  m.def("crc32c_unmask", &crc32c_unmask);
  m.def("snappy_uncompress", [](py::bytes b) {
    std::string_view sv = b;
    return py::bytes(snappy_uncompress(reinterpret_cast<const uint8_t*>(sv.data()), sv.size()));
  });
  m.def("read_sstable", [](py::bytes data, bool verify) {
    std::string file = data;
    std::vector<std::pair<std::string, std::string>> kv;
    {
      py::gil_scoped_release nogil;
      kv = read_sstable(file, verify);
    }
    py::list out;
    for (auto& e : kv) out.append(py::make_tuple(py::bytes(e.first), py::bytes(e.second)));
    return out;
  }, py::arg("data"), py::arg("verify_crc") = true);

  py::class_<Batch>(m, "Batch")
      .def_readonly("id", &Batch::id)
      .def_readonly("n_real", &Batch::n_real)
      .def_readonly("bucket", &Batch::bucket)
      .def_readonly("tickets", &Batch::tickets)
      .def_readonly("first_item", &Batch::first_item)
      .def_readonly("n_items", &Batch::n_items)
      .def_property_readonly("dev_src", [](const Batch& b) {
        std::vector<uintptr_t> v;
        for (auto p : b.dev_src) v.push_back(reinterpret_cast<uintptr_t>(p));
        return v;
      })
      .def_readonly("oldest_enqueue_us", &Batch::oldest_enqueue_us);

  // shared holder: the native gRPC front-end's routes keep a signature's batcher alive
  py::class_<DynamicBatcher, std::shared_ptr<DynamicBatcher>>(m, "DynamicBatcher")
      .def(py::init([](int max_batch_size, int64_t batch_timeout_us, int max_enqueued_batches,
                       std::vector<int> allowed_batch_sizes, size_t item_bytes, int out_cols, int copy_threads) {
             BatcherOptions o;
             o.copy_threads = copy_threads;
             o.max_batch_size = max_batch_size;
             o.batch_timeout_us = batch_timeout_us;
             o.max_enqueued_batches = max_enqueued_batches;
             o.allowed_batch_sizes = allowed_batch_sizes;
             o.item_bytes = item_bytes;
             o.out_cols = out_cols;
             return std::make_shared<DynamicBatcher>(o);
           }),
           py::arg("max_batch_size") = 32, py::arg("batch_timeout_us") = 2000,
           py::arg("max_enqueued_batches") = 1000, py::arg("allowed_batch_sizes") = std::vector<int>{},
           py::arg("item_bytes") = 0, py::arg("out_cols") = 0, py::arg("copy_threads") = 4)
      // `data` must stay alive until wait() returns (the Python wrapper holds it).
      .def("submit", [](DynamicBatcher& b, py::buffer data, int n_items, int64_t deadline_us) {
        py::buffer_info info = data.request();
        const size_t need = size_t(n_items) * b.options().item_bytes;
        if (size_t(info.size) * size_t(info.itemsize) < need) throw std::invalid_argument("payload smaller than n_items*item_bytes");
        return b.submit(reinterpret_cast<const uint8_t*>(info.ptr), n_items, deadline_us);
      })
      // device-resident payload (an address in device memory, e.g. a GPU-resized image batch):
      // only native executors whose backend has issue_dev can run such batches
      .def("submit_device", [](DynamicBatcher& b, uintptr_t ptr, int n_items, int64_t deadline_us) {
        if (!ptr) throw std::invalid_argument("null device payload");
        return b.submit(reinterpret_cast<const uint8_t*>(ptr), n_items, deadline_us, true);
      })
      // `out` may be larger than the ticket's n_items*out_cols floats, never smaller: a short
      // buffer gets ST_ERROR and is left untouched (the C++ side checks the size it is given)
      .def("wait", [](DynamicBatcher& b, int64_t ticket, py::array_t<float, py::array::c_style> out) {
        float* p = out.mutable_data();
        const size_t cap = size_t(out.size());
        py::gil_scoped_release nogil;
        return b.wait(ticket, p, cap);
      })
      .def("next_batch", [](DynamicBatcher& b, uintptr_t staging, int64_t poll_us, bool eager) -> py::object {
        Batch batch;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = b.next_batch(reinterpret_cast<uint8_t*>(staging), poll_us, &batch, eager);
        }
        if (!ok) return py::none();
        return py::cast(batch);
      }, py::arg("staging"), py::arg("poll_us"), py::arg("eager") = false)
      .def("finish", [](DynamicBatcher& b, const Batch& batch, uintptr_t results, int status) {
        py::gil_scoped_release nogil;
        b.finish(batch, reinterpret_cast<const float*>(results), status);
      })
      .def("bucket_for", &DynamicBatcher::bucket_for)
      .def("shutdown", &DynamicBatcher::shutdown)
      .def("stats", [](const DynamicBatcher& b) {
        BatcherStats s = b.stats();
        py::dict d;
        d["submitted"] = s.submitted; d["completed"] = s.completed; d["expired"] = s.expired;
        d["rejected"] = s.rejected; d["batches"] = s.batches; d["items"] = s.items;
        d["padded_items"] = s.padded_items; d["queue_items"] = s.queue_items;
        return d;
      });
  // ---- native gRPC front-end (runtime/grpc_front.h) + the native load generator
  py::class_<GrpcFront, std::unique_ptr<GrpcFront, FrontDeleter>>(m, "GrpcFront")
      // slow(path: str, message: bytes, deadline_us: int) -> (code, message, body: bytes, [(k, v)])
      .def(py::init([](const std::string& host, int port, int io_threads, int slow_threads, py::function slow,
                       size_t max_recv_bytes, bool reuse_port) {
             auto fn = std::make_shared<py::function>(std::move(slow));
             SlowFn cb = [fn](const std::string& path, const std::string& msg, int64_t deadline_us) {
               py::gil_scoped_acquire gil;
               SlowReply r;
               py::tuple t = (*fn)(path, py::bytes(msg), deadline_us);
               r.code = t[0].cast<int>();
               r.message = t[1].cast<std::string>();
               r.body = t[2].cast<std::string>();
               for (auto kv : t[3].cast<py::list>()) {
                 auto p = kv.cast<py::tuple>();
                 r.meta.emplace_back(p[0].cast<std::string>(), p[1].cast<std::string>());
               }
               return r;
             };
             // built with the GIL held: a constructor that throws drops the callable safely (its
             // threads never wait on Python before a request arrives)
             return std::unique_ptr<GrpcFront, FrontDeleter>(
                 new GrpcFront(host, port, io_threads, slow_threads, std::move(cb), max_recv_bytes, reuse_port));
           }),
           py::arg("host"), py::arg("port"), py::arg("io_threads") = 2, py::arg("slow_threads") = 4, py::arg("slow"),
           py::arg("max_recv_bytes") = size_t(64) << 20, py::arg("reuse_port") = true)
      .def_property_readonly("port", &GrpcFront::port)
      .def("set_route", [](GrpcFront& f, const std::string& model, const std::string& signature, int64_t version,
                           const std::string& input_key, const std::string& output_key, int dtype, int image,
                           int out_cols, std::shared_ptr<DynamicBatcher> batcher, std::shared_ptr<DynamicBatcher> u8) {
             FrontRoute r;
             r.model = model; r.signature = signature; r.version = version; r.input_key = input_key;
             r.output_key = output_key; r.dtype = dtype; r.image = image; r.out_cols = out_cols;
             r.batcher = std::move(batcher); r.u8 = std::move(u8);
             f.set_route(std::move(r));
           },
           py::arg("model"), py::arg("signature"), py::arg("version"), py::arg("input_key"), py::arg("output_key"),
           py::arg("dtype"), py::arg("image"), py::arg("out_cols"), py::arg("batcher"), py::arg("u8") = nullptr)
      .def("clear_routes", &GrpcFront::clear_routes)
      .def("stop", &GrpcFront::stop, py::call_guard<py::gil_scoped_release>())
      .def("stats", [](const GrpcFront& f) {
        const FrontStats s = f.stats();
        py::dict d;
        d["fast_ok"] = s.fast_ok; d["fast_err"] = s.fast_err; d["slow"] = s.slow; d["exact_u8"] = s.exact_u8;
        d["connections"] = s.connections; d["open_connections"] = s.open_connections;
        py::dict codes;
        for (int i = 0; i < 17; ++i)
          if (s.by_code[i]) codes[py::int_(i)] = s.by_code[i];
        d["by_code"] = codes;
        py::list lat;
        for (int i = 0; i <= kFrontLatBuckets; ++i) lat.append(s.lat[i]);
        d["lat_counts"] = lat;
        d["lat_sum_ms"] = s.lat_sum_ms;
        py::list wc;
        for (int i = 0; i < FrontStats::kMaxWorkers; ++i) wc.append(s.worker_calls[i]);
        while (py::len(wc) && wc[py::len(wc) - 1].cast<int64_t>() == 0) wc.attr("pop")();
        d["worker_calls"] = wc;
        return d;
      });
  m.def("grpc_percent_encode", &grpc_percent_encode);
  m.def("http2_available", [] {
    std::string why;
    const bool ok = h2::api(&why) != nullptr;
    return py::make_tuple(ok, why);
  });
  m.def("grpc_load", [](const std::string& host, int port, const std::string& path, py::bytes message, int conns,
                        int streams, double seconds, double warm_s, double timeout_s, bool raw_frame) {
          std::string msg = message;
          LoadResult r;
          {
            py::gil_scoped_release nogil;
            r = grpc_load(host, port, path, msg, conns, streams, seconds, warm_s, timeout_s, raw_frame);
          }
          py::dict d;
          d["ok"] = r.ok; d["failed"] = r.failed; d["seconds"] = r.seconds; d["error"] = r.error;
          d["lat_ms"] = r.lat_ms;
          py::dict codes;
          for (auto& kv : r.codes) codes[py::int_(kv.first)] = kv.second;
          d["codes"] = codes;
          return d;
        }, py::arg("host"), py::arg("port"), py::arg("path"), py::arg("message"), py::arg("conns") = 4,
        py::arg("streams") = 8, py::arg("seconds") = 5.0, py::arg("warm_s") = 1.0, py::arg("timeout_s") = 30.0,
        py::arg("raw_frame") = false);

  // ---- native batch executor (executor.h) + the fake device backend used by CPU tests
  py::class_<ExecGroup>(m, "ExecGroup")
      .def(py::init<>())
      .def("healthy", &ExecGroup::healthy);
  py::class_<FakeBackend>(m, "FakeBackend")
      .def(py::init<int, size_t, int, int, int64_t, int>(), py::arg("nslots"), py::arg("item_bytes"),
           py::arg("max_batch"), py::arg("out_cols"), py::arg("latency_us") = 0, py::arg("fail_every") = 0)
      .def("api_ptr", [](FakeBackend& f) { return reinterpret_cast<uintptr_t>(&f.api); })
      .def_readonly("issued", &FakeBackend::issued)
      .def_readonly("dev_pieces", &FakeBackend::dev_pieces);
  py::class_<Executor>(m, "Executor")
      // `backend`: any object with api_ptr() -> address of its kdl_exec_backend (kdl._C.HipExecBackend,
      // FakeBackend). The executor keeps the batcher, the backend and the group alive (keep_alive):
      // its C++ thread uses all three until stop() joins it in the executor's destructor, whatever
      // order Python tears objects down in
      .def(py::init([](DynamicBatcher* b, py::object backend, ExecGroup* g, const std::string& name, bool eager,
                       int max_failures, int64_t poll_us, int fail_batches, int64_t delay_us, int trace_ring) {
             ExecOptions o;
             o.name = name; o.eager = eager; o.max_failures = max_failures; o.poll_us = poll_us;
             o.fail_batches = fail_batches; o.delay_us = delay_us; o.trace_ring = trace_ring;
             const auto ptr = backend.attr("api_ptr")().cast<uintptr_t>();
             return new Executor(b, reinterpret_cast<const kdl_exec_backend*>(ptr), g, o);
           }),
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>(), py::keep_alive<1, 4>(),
           py::arg("batcher"), py::arg("backend"), py::arg("group"), py::arg("name") = "exec",
           py::arg("eager") = true, py::arg("max_failures") = 3, py::arg("poll_us") = 100000,
           py::arg("fail_batches") = 0, py::arg("delay_us") = 0, py::arg("trace_ring") = 256)
      .def("start", &Executor::start)
      .def("stop", [](Executor& e) { py::gil_scoped_release nogil; e.stop(); })
      .def("healthy", &Executor::healthy)
      .def("running", &Executor::running)
      .def("stats", [](const Executor& e) {
        const ExecStats s = e.stats();
        py::dict d;
        d["batches"] = s.batches; d["items"] = s.items; d["padded_items"] = s.padded_items;
        d["failed_batches"] = s.failed_batches; d["healthy"] = s.healthy;
        py::dict st;
        py::list le;
        for (int i = 0; i < N_BUCKETS; ++i) le.append(kBucketsMs[i]);
        for (int k = 0; k < N_STAGES; ++k) {
          py::dict h;
          h["count"] = s.hist[k].count; h["sum_ms"] = s.hist[k].sum_ms;
          py::list bk;
          for (int i = 0; i < N_BUCKETS; ++i) bk.append(s.hist[k].buckets[i]);
          h["buckets"] = bk;
          st[exec_stage_name(k)] = h;
        }
        d["stages"] = st;
        d["le_ms"] = le;
        return d;
      })
      .def("recent", [](const Executor& e, int n) {
        py::list out;
        for (const BatchTrace& t : e.recent(n)) {
          py::dict d;
          d["batch_id"] = t.batch_id; d["n_real"] = t.n_real; d["bucket"] = t.bucket; d["slot"] = t.slot;
          d["status"] = t.status; d["oldest_enqueue_us"] = t.oldest_enqueue_us; d["formed_us"] = t.formed_us;
          d["copied_us"] = t.copied_us; d["issued_us"] = t.issued_us; d["completed_us"] = t.completed_us;
          d["finished_us"] = t.finished_us; d["h2d_ms"] = t.h2d_ms; d["forward_ms"] = t.forward_ms;
          d["d2h_ms"] = t.d2h_ms;
          out.append(d);
        }
        return out;
      }, py::arg("n") = 64);

  // ---- loopback data-parallel platform (runtime/dp_loop.h): the SAME leader / follower state
  // machine as the RCCL path (runtime/dp_core.h), over threads and host memory, for CPU tests
  m.def("loop_unique_id", &loop::unique_id);
  py::class_<loop::Comm>(m, "LoopComm")
      .def(py::init<const std::string&, int, int>(), py::arg("id"), py::arg("nranks"), py::arg("rank"))
      .def_property_readonly("rank", &loop::Comm::rank)
      .def_property_readonly("size", &loop::Comm::size)
      .def("kill", &loop::Comm::kill)
      .def("abort", &loop::Comm::abort)
      .def("error", &loop::Comm::error);
  py::class_<loop::Device>(m, "LoopDevice")
      .def(py::init<int, int, size_t, int, int, std::vector<int>, int, int64_t>(), py::arg("rank"), py::arg("nslots"),
           py::arg("item_bytes"), py::arg("max_batch"), py::arg("out_cols"), py::arg("buckets"), py::arg("version") = 0,
           py::arg("latency_us") = 0)
      .def("api_ptr", [](const loop::Device& d) { return reinterpret_cast<uintptr_t>(d.api()); })
      .def_property_readonly("forwards", &loop::Device::forwards)
      .def("fail_issues", &loop::Device::fail_issues, py::arg("n"))
      .def_static("logit", &loop::Device::logit);
  py::class_<LoopDpLeader>(m, "LoopDpLeader")
      .def(py::init([](loop::Device* local, loop::Comm* sc, loop::Comm* ga, std::vector<int> buckets, double timeout_s,
                       double ping_s) { return new LoopDpLeader(local, sc, ga, std::move(buckets), timeout_s, ping_s); }),
           py::arg("local"), py::arg("scatter"), py::arg("gather"), py::arg("rank_buckets"), py::arg("timeout_s") = 10.0,
           py::arg("ping_s") = 0.0, py::keep_alive<1, 2>(), py::keep_alive<1, 3>(), py::keep_alive<1, 4>())
      .def("api_ptr", [](const LoopDpLeader& l) { return reinterpret_cast<uintptr_t>(l.api()); })
      .def_property_readonly("world", &LoopDpLeader::world)
      .def_property_readonly("steps", &LoopDpLeader::steps)
      .def_property_readonly("broken", &LoopDpLeader::broken)
      .def("send_ctrl", [](LoopDpLeader& l, int cmd, int version) {
        py::gil_scoped_release nogil;
        return l.send_ctrl(cmd, version);
      })
      .def("ping", [](LoopDpLeader& l) {
        py::gil_scoped_release nogil;
        return l.ping();
      });
  py::class_<LoopDpFollower>(m, "LoopDpFollower")
      .def(py::init([](loop::Device* local, loop::Comm* sc, loop::Comm* ga) { return new LoopDpFollower(local, sc, ga); }),
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>(), py::keep_alive<1, 4>())
      .def_property_readonly("steps", &LoopDpFollower::steps)
      // serve until DP_STOP / DP_RELOAD; returns (cmd, version, seq); raises RuntimeError when the
      // leader is silent for liveness_s or a communicator failed
      .def("run", [](LoopDpFollower& f, double liveness_s) {
        DpCtrl c{};
        {
          py::gil_scoped_release nogil;
          c = f.run(liveness_s);
        }
        return std::make_tuple(c.cmd, c.version, c.seq);
      }, py::arg("liveness_s") = 30.0);
  m.attr("DP_STOP") = int(DP_STOP);
  m.attr("DP_BATCH") = int(DP_BATCH);
  m.attr("DP_RELOAD") = int(DP_RELOAD);
  m.attr("DP_PING") = int(DP_PING);

  m.attr("ST_OK") = int(ST_OK);
  m.attr("ST_DEADLINE") = int(ST_DEADLINE);
  m.attr("ST_SHUTDOWN") = int(ST_SHUTDOWN);
  m.attr("ST_ERROR") = int(ST_ERROR);
  m.attr("ST_QUEUE_FULL") = int(ST_QUEUE_FULL);
}
