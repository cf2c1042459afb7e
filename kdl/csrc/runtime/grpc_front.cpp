#include "grpc_front.h"

#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "h2.h"
#include "tfproto.h"

// AVX2 clone picked at load time (an ifunc). Not under ThreadSanitizer: the ifunc resolver runs
// during relocation, before the TSAN runtime is up, and instrumented it crashes the process
#if defined(__SANITIZE_THREAD__)
#define KDL_SIMD_CLONES
#elif defined(__has_feature)
#if __has_feature(thread_sanitizer)
#define KDL_SIMD_CLONES
#endif
#endif
#ifndef KDL_SIMD_CLONES
#define KDL_SIMD_CLONES __attribute__((target_clones("avx2", "default")))
#endif

namespace kdl {

KDL_SIMD_CLONES bool f32_to_u8_exact(const float* __restrict x,
                                                                       uint8_t* __restrict u, size_t n) {
  // branch-free and vectorized (round 4's std::nearbyint + float min/max form stayed scalar:
  // 1.2 ms per 299x299x3 image, profiles/serve_f32_exact_r5.txt); blocks allow an early exit
  const size_t B = 4096;
  for (size_t i0 = 0; i0 < n; i0 += B) {
    const size_t i1 = std::min(n, i0 + B);
    int bad = 0;
    for (size_t i = i0; i < i1; ++i) {
      int r = (int)((x[i] + 1.0f) * 127.5f + 0.5f);   // NaN / out of range -> INT_MIN: clamped, then mismatches
      r = r < 0 ? 0 : r > 255 ? 255 : r;
      bad |= (float)r / 127.5f - 1.0f != x[i];       // rebuilt exactly as the gateway computed it
      u[i] = (uint8_t)r;
    }
    if (bad) return false;
  }
  return true;
}

std::string grpc_percent_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  o.reserve(s.size());
  for (unsigned char ch : s) {
    if (ch >= 0x20 && ch <= 0x7e && ch != '%') {
      o.push_back(char(ch));
    } else {
      o.push_back('%');
      o.push_back(hex[ch >> 4]);
      o.push_back(hex[ch & 15]);
    }
  }
  return o;
}

namespace {

constexpr double kLatMs[kFrontLatBuckets] = {0.5, 1,  2,  3,   5,   7.5,  10,   15,   20,   30,
                                             50,  75, 100, 200, 500, 1000, 2000, 5000, 20000};
const std::string kPredictPath = "/tensorflow.serving.PredictionService/Predict";
enum : int { G_OK = 0, G_DEADLINE = 4, G_RESOURCE = 8, G_UNIMPLEMENTED = 12, G_INTERNAL = 13, G_UNAVAILABLE = 14 };
constexpr uint64_t kListenTag = ~uint64_t(0), kWakeTag = ~uint64_t(0) - 1;
constexpr int32_t kStreamWindow = 8 << 20, kConnWindow = 64 << 20, kMaxFrame = 1 << 20;

uint32_t be32(const uint8_t* p) { return uint32_t(p[0]) << 24 | uint32_t(p[1]) << 16 | uint32_t(p[2]) << 8 | p[3]; }

std::string grpc_frame(const std::string& msg) {
  std::string f(5, '\0');
  const uint32_t n = uint32_t(msg.size());
  f[1] = char(n >> 24), f[2] = char(n >> 16), f[3] = char(n >> 8), f[4] = char(n);
  return f + msg;
}

// grpc-timeout header ("<digits><unit>", gRPC HTTP/2 protocol) -> microseconds, 0 = none
int64_t parse_grpc_timeout(const std::string& v) {
  if (v.size() < 2 || v.size() > 9) return 0;
  int64_t n = 0;
  for (size_t i = 0; i + 1 < v.size(); ++i) {
    if (v[i] < '0' || v[i] > '9') return 0;
    n = n * 10 + (v[i] - '0');
  }
  switch (v.back()) {
    case 'H': return n * 3600000000LL;
    case 'M': return n * 60000000LL;
    case 'S': return n * 1000000LL;
    case 'm': return n * 1000LL;
    case 'u': return n;
    case 'n': return std::max<int64_t>(1, n / 1000);
    default: return 0;
  }
}

// one RPC (one HTTP/2 stream)
struct Call {
  uint64_t conn = 0;
  int32_t stream = 0;
  int worker = 0;
  std::string path, timeout;
  std::string body;                      // framed request: 5-byte gRPC prefix + message
  int64_t t0_us = 0, deadline_us = 0;
  std::vector<uint8_t> u8;               // exact-u8 copy of an f32 payload (fast path)
  bool fast = false;
  std::shared_ptr<const FrontRoute> route;   // fast path: the route that served it
  std::vector<float> rows;               // fast path: result rows, turned into `resp` by the worker
  int64_t n = 0;
  int code = 0;                          // reply: grpc status, message, framed response, metadata
  std::string message, resp;
  std::vector<std::pair<std::string, std::string>> meta;
  size_t sent = 0;
  bool rejected = false;                 // answered while its body was still arriving (size caps)
  // request bytes this call holds against the front's budget, returned when the call dies
  std::shared_ptr<std::atomic<int64_t>> budget;
  int64_t held = 0;
  ~Call() {
    if (budget && held) budget->fetch_sub(held, std::memory_order_relaxed);
  }
};
using CallP = std::shared_ptr<Call>;

// Completed calls travel to their connection's worker through here. Shared with the batcher
// callbacks, so it outlives the front: a callback arriving after stop() finds `closed`.
struct Mailbox {
  struct Box {
    std::mutex mu;
    std::vector<CallP> q;
    int efd = -1;
  };
  std::vector<std::unique_ptr<Box>> box;
  std::atomic<bool> closed{false};
  ~Mailbox() {
    for (auto& b : box)
      if (b->efd >= 0) ::close(b->efd);
  }
  void post(CallP c) {
    if (closed.load(std::memory_order_acquire)) return;
    Box& b = *box[size_t(c->worker)];
    bool wake;
    {
      std::lock_guard<std::mutex> lk(b.mu);
      wake = b.q.empty();                // a non-empty box has a wake-up pending already
      b.q.push_back(std::move(c));
    }
    if (wake) {
      const uint64_t one = 1;
      (void)!::write(b.efd, &one, sizeof one);
    }
  }
};

struct Worker;

struct Conn {
  uint64_t id = 0;
  int fd = -1;
  Worker* w = nullptr;
  h2::session* s = nullptr;
  std::unordered_map<int32_t, CallP> calls;   // open streams
  std::string out;                           // produced bytes the socket has not taken yet
  size_t out_off = 0;
  bool pollout = false;
  // streams answered before their request ended: RST_STREAM(NO_ERROR) once the answer's
  // HEADERS are serialized (queued together, nghttp2 may emit the RST first and the client
  // would see no status)
  std::vector<int32_t> rst_after;
};

}  // namespace

struct GrpcFront::Impl {
  const h2::Api* H = nullptr;
  h2::callbacks* cbs = nullptr;
  SlowFn slow;
  int port = 0;
  // request size caps (advisor r5): one message at most max_recv bytes; all request bodies
  // held by the front (receiving, queued for the slow path, waiting in a batcher) at most
  // max_held bytes -- past either the stream is answered RESOURCE_EXHAUSTED and its data dropped
  size_t max_recv = size_t(64) << 20;
  int64_t max_held = int64_t(1) << 30;
  std::shared_ptr<std::atomic<int64_t>> held = std::make_shared<std::atomic<int64_t>>(0);
  std::vector<std::unique_ptr<Worker>> workers;
  std::shared_ptr<Mailbox> mail = std::make_shared<Mailbox>();
  std::atomic<bool> stopping{false};
  std::mutex stop_mu;
  bool stopped = false;

  using RouteMap = std::unordered_map<std::string, std::shared_ptr<const FrontRoute>>;
  mutable std::mutex rmu;
  std::shared_ptr<const RouteMap> routes = std::make_shared<RouteMap>();

  std::mutex qmu;
  std::condition_variable qcv;
  std::deque<CallP> sq;
  bool sstop = false;
  std::vector<std::thread> slow_threads;

  mutable std::mutex stmu;
  FrontStats st;

  void run(Worker* w);
  void accept_all(Worker* w);
  void on_readable(Worker* w, Conn* c);
  bool flush(Worker* w, Conn* c);
  void close_conn(Worker* w, Conn* c);
  void want_out(Worker* w, Conn* c, bool on);
  void dispatch(Worker* w, const CallP& call);
  bool fast_predict(Worker* w, const CallP& call);
  void answer(Worker* w, const CallP& call);
  void slow_loop();
  std::shared_ptr<const FrontRoute> find_route(const std::string& model, const std::string& sig) const {
    std::shared_ptr<const RouteMap> m;
    {
      std::lock_guard<std::mutex> lk(rmu);
      m = routes;
    }
    auto it = m->find(model + '\0' + sig);
    return it == m->end() ? nullptr : it->second;
  }
};

namespace {

struct Worker {
  GrpcFront::Impl* impl = nullptr;
  int idx = 0, ep = -1, lfd = -1, efd = -1;
  std::thread th;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns;
  uint64_t next = 1;
  std::vector<CallP> local;              // answers made inside nghttp2 callbacks, sent after them
  std::vector<uint8_t> rbuf = std::vector<uint8_t>(size_t(1) << 18);
};

void set_error(Call& c, int code, std::string msg) {
  c.code = code;
  c.message = std::move(msg);
  c.resp.clear();
}

// ---- nghttp2 server callbacks (user_data = the Conn) ----
// Every body is guarded: an exception unwinding through nghttp2's C frames would terminate the
// process (and every GPU slot's batches with it); a failing callback fails its connection only.
#define KDL_CB_GUARD(...)                    \
  try {                                      \
    __VA_ARGS__                              \
  } catch (...) {                            \
    return h2::ERR_CALLBACK_FAILURE;         \
  }                                          \
  return 0;

// answer a stream before its request is complete and drop whatever else it sends
void reject_early(Conn* c, const CallP& call, int code, std::string msg) {
  call->rejected = true;
  set_error(*call, code, std::move(msg));
  std::string().swap(call->body);
  if (call->budget && call->held) call->budget->fetch_sub(call->held, std::memory_order_relaxed);
  call->held = 0;
  c->w->local.push_back(call);
}

int cb_begin_headers(h2::session*, const h2::frame_hd* f, void* ud) {
  KDL_CB_GUARD({
    if (f->type != h2::FRAME_HEADERS) return 0;
    Conn* c = static_cast<Conn*>(ud);
    if (c->calls.count(f->stream_id)) return 0;   // trailers of a known stream
    auto call = std::make_shared<Call>();
    call->conn = c->id;
    call->stream = f->stream_id;
    call->worker = c->w->idx;
    call->t0_us = now_us();
    c->calls.emplace(f->stream_id, std::move(call));
    return 0;
  })
}

int cb_header(h2::session*, const h2::frame_hd* f, const uint8_t* n, size_t nl, const uint8_t* v, size_t vl, uint8_t,
              void* ud) {
  KDL_CB_GUARD({
    if (f->type != h2::FRAME_HEADERS) return 0;
    Conn* c = static_cast<Conn*>(ud);
    auto it = c->calls.find(f->stream_id);
    if (it == c->calls.end()) return 0;
    const std::string_view name(reinterpret_cast<const char*>(n), nl);
    if (name == ":path") it->second->path.assign(reinterpret_cast<const char*>(v), vl);
    else if (name == "grpc-timeout") it->second->timeout.assign(reinterpret_cast<const char*>(v), vl);
    return 0;
  })
}

int cb_data_chunk(h2::session*, uint8_t, int32_t sid, const uint8_t* d, size_t len, void* ud) {
  KDL_CB_GUARD({
    Conn* c = static_cast<Conn*>(ud);
    auto it = c->calls.find(sid);
    if (it == c->calls.end() || it->second->rejected) return 0;
    const CallP& call = it->second;
    GrpcFront::Impl& I = *c->w->impl;
    std::string& b = call->body;
    // the body grows by the bytes that arrived; the client's length prefix is checked against
    // the cap before it sizes any allocation
    if (b.size() + len > I.max_recv + 5) {
      reject_early(c, call, G_RESOURCE, "SERVER: Received message larger than max (" +
                   std::to_string(b.size() + len - 5) + " vs. " + std::to_string(I.max_recv) + ")");
      return 0;
    }
    if (I.held->fetch_add(int64_t(len), std::memory_order_relaxed) + int64_t(len) > I.max_held) {
      I.held->fetch_sub(int64_t(len), std::memory_order_relaxed);
      reject_early(c, call, G_RESOURCE, "server request memory budget exhausted");
      return 0;
    }
    if (!call->budget) call->budget = I.held;
    call->held += int64_t(len);
    const bool first = b.size() < 5;
    b.append(reinterpret_cast<const char*>(d), len);
    if (first && b.size() >= 5) {        // the message length is known
      if (uint8_t(b[0]) == 1) {
        reject_early(c, call, G_UNIMPLEMENTED, "compressed gRPC messages are not supported");
        return 0;
      }
      const uint32_t m = be32(reinterpret_cast<const uint8_t*>(b.data()) + 1);
      if (m > I.max_recv) {
        reject_early(c, call, G_RESOURCE, "SERVER: Received message larger than max (" + std::to_string(m) + " vs. " +
                     std::to_string(I.max_recv) + ")");
        return 0;
      }
      b.reserve(size_t(5) + m);          // m <= max_recv: one allocation for the rest
    }
    return 0;
  })
}

int cb_frame_recv(h2::session*, const h2::frame_hd* f, void* ud) {
  KDL_CB_GUARD({
    if ((f->type != h2::FRAME_DATA && f->type != h2::FRAME_HEADERS) || !(f->flags & h2::FLAG_END_STREAM)) return 0;
    Conn* c = static_cast<Conn*>(ud);
    auto it = c->calls.find(f->stream_id);
    if (it != c->calls.end() && !it->second->rejected) c->w->impl->dispatch(c->w, it->second);
    return 0;
  })
}

int cb_stream_close(h2::session*, int32_t sid, uint32_t, void* ud) {
  KDL_CB_GUARD({
    static_cast<Conn*>(ud)->calls.erase(sid);
    return 0;
  })
}

ssize_t cb_read_resp(h2::session* s, int32_t sid, uint8_t* buf, size_t len, uint32_t* flags, h2::data_source* src,
                     void* ud) {
  KDL_CB_GUARD({
    Call* call = static_cast<Call*>(src->ptr);
    const size_t n = std::min(len, call->resp.size() - call->sent);
    std::memcpy(buf, call->resp.data() + call->sent, n);
    call->sent += n;
    if (call->sent == call->resp.size()) {
      *flags |= h2::DATA_FLAG_EOF | h2::DATA_FLAG_NO_END_STREAM;
      static const std::string k = "grpc-status", v = "0";
      const h2::nv tr = h2::make_nv(k, v);
      static_cast<Conn*>(ud)->w->impl->H->submit_trailer(s, sid, &tr, 1);
    }
    return ssize_t(n);
  })
}
#undef KDL_CB_GUARD

}  // namespace

// ---------------------------------------------------------------- request handling
void GrpcFront::Impl::dispatch(Worker* w, const CallP& call) {
  const std::string& b = call->body;
  if (b.size() < 5 || uint8_t(b[0]) > 1 || be32(reinterpret_cast<const uint8_t*>(b.data()) + 1) != b.size() - 5) {
    set_error(*call, G_INTERNAL, "malformed gRPC request message (one length-prefixed message expected)");
    w->local.push_back(call);
    return;
  }
  if (b[0] == 1) {
    set_error(*call, G_UNIMPLEMENTED, "compressed gRPC messages are not supported");
    w->local.push_back(call);
    return;
  }
  if (!call->timeout.empty()) {
    const int64_t t = parse_grpc_timeout(call->timeout);
    if (t > 0 && t < int64_t(1e14)) call->deadline_us = call->t0_us + t;   // > 1e8 s: none (as grpc_server.py)
  }
  {
    std::lock_guard<std::mutex> lk(stmu);
    ++st.worker_calls[std::min(w->idx, FrontStats::kMaxWorkers - 1)];
  }
  if (call->path == kPredictPath && fast_predict(w, call)) return;
  {
    std::lock_guard<std::mutex> lk(stmu);
    ++st.slow;
  }
  {
    std::lock_guard<std::mutex> lk(qmu);
    sq.push_back(call);
  }
  qcv.notify_one();
}

bool GrpcFront::Impl::fast_predict(Worker* w, const CallP& call) {
  const uint8_t* msg = reinterpret_cast<const uint8_t*>(call->body.data()) + 5;
  const size_t len = call->body.size() - 5;
  PredictRequestView v;
  try {
    v = parse_predict_request(msg, len);
  } catch (const std::exception&) {
    return false;                        // the servicer words the error
  }
  if (!v.spec.version_label.empty() || v.inputs.size() != 1) return false;
  const std::string sig = v.spec.signature_name.empty() ? "serving_default" : v.spec.signature_name;
  std::shared_ptr<const FrontRoute> r = find_route(v.spec.name, sig);
  if (!r || !r->batcher || (v.spec.version >= 0 && v.spec.version != r->version)) return false;
  const TensorView& t = v.inputs[0].second;
  if (v.inputs[0].first != r->input_key || !t.has_content || t.dtype != r->dtype || t.dims.size() != 4) return false;
  const int64_t n = t.dims[0], S = r->image;
  if (t.dims[1] != S || t.dims[2] != S || t.dims[3] != 3 || n < 1 || n > r->batcher->options().max_batch_size)
    return false;
  const size_t pix = size_t(S) * size_t(S) * 3;
  if (t.content_size != size_t(n) * pix * (r->dtype == 1 ? 4 : 1)) return false;
  for (const auto& f : v.output_filter)
    if (f != r->output_key) return false;
  const uint8_t* payload = msg + t.content_offset;
  std::shared_ptr<DynamicBatcher> b = r->batcher;
  if (r->dtype == 1 && r->u8 && n <= r->u8->options().max_batch_size) {
    call->u8.resize(size_t(n) * pix);
    if (f32_to_u8_exact(reinterpret_cast<const float*>(payload), call->u8.data(), call->u8.size())) {
      payload = call->u8.data();
      b = r->u8;
      std::lock_guard<std::mutex> lk(stmu);
      ++st.exact_u8;
    }
  }
  call->fast = true;
  call->route = r;
  call->n = n;
  std::shared_ptr<Mailbox> mail = this->mail;
  const int64_t tk = b->submit_async(payload, int(n), call->deadline_us,
      [call, mail](int status, const float* rows, size_t nf) {
        // runs on the executor thread that finished the batch: copy the rows only; the
        // response is built by the connection's worker (answer), off the GPU issue path
        if (status == ST_OK && rows && nf == size_t(call->n) * size_t(call->route->out_cols)) {
          call->rows.assign(rows, rows + nf);
          call->code = G_OK;
        } else if (status == ST_DEADLINE) {    // serving/backend.py SignatureRunner._run's wording
          set_error(*call, G_DEADLINE, "deadline exceeded while queued for batching");
        } else {
          set_error(*call, status == ST_ERROR || status == ST_OK ? G_INTERNAL : G_UNAVAILABLE,
                    "batch failed (status " + std::to_string(status == ST_OK ? int(ST_ERROR) : status) + ")");
        }
        mail->post(call);
      });
  if (tk > 0) return true;
  call->fast = false;
  if (-tk == ST_QUEUE_FULL) {
    set_error(*call, G_RESOURCE, "batcher rejected request (status " + std::to_string(-tk) + ")");
    call->fast = true;
    w->local.push_back(call);
    return true;
  }
  return false;                          // shut down (a version change): the servicer answers
}

void GrpcFront::Impl::answer(Worker* w, const CallP& call) {
  auto ci = w->conns.find(call->conn);
  if (ci == w->conns.end()) return;      // the client went away
  Conn* c = ci->second.get();
  auto si = c->calls.find(call->stream);
  if (si == c->calls.end() || si->second != call) return;   // stream reset
  if (call->code == G_OK && call->route && call->resp.empty()) {   // fast path: build the response here
    const FrontRoute& r = *call->route;
    ModelSpecView spec;
    spec.name = r.model;
    spec.version = r.version;
    spec.signature_name = r.signature;
    const OutputTensor o{r.output_key, {call->n, int64_t(r.out_cols)}, call->rows.data()};
    call->resp = grpc_frame(build_predict_response({o}, spec));
  }
  if (call->fast) {
    const double ms = (now_us() - call->t0_us) * 1e-3;
    std::lock_guard<std::mutex> lk(stmu);
    ++(call->code == G_OK ? st.fast_ok : st.fast_err);
    ++st.by_code[std::min(16, std::max(0, call->code))];
    st.lat[std::lower_bound(kLatMs, kLatMs + kFrontLatBuckets, ms) - kLatMs] += 1;
    st.lat_sum_ms += ms;
  }
  static const std::string ks = ":status", v200 = "200", kct = "content-type", vct = "application/grpc",
                           kgs = "grpc-status", kgm = "grpc-message";
  std::vector<h2::nv> nva{h2::make_nv(ks, v200), h2::make_nv(kct, vct)};
  for (const auto& m : call->meta) nva.push_back(h2::make_nv(m.first, m.second));
  if (call->code == G_OK) {
    h2::data_provider dp;
    dp.source.ptr = call.get();          // alive in c->calls until the stream closes
    dp.read_callback = cb_read_resp;
    if (H->submit_response(c->s, call->stream, nva.data(), nva.size(), &dp) != 0)
      H->submit_rst_stream(c->s, 0, call->stream, h2::INTERNAL_ERROR);
  } else {                               // Trailers-Only response
    const std::string code = std::to_string(call->code), msg = grpc_percent_encode(call->message);
    nva.push_back(h2::make_nv(kgs, code));
    if (!msg.empty()) nva.push_back(h2::make_nv(kgm, msg));
    if (H->submit_response(c->s, call->stream, nva.data(), nva.size(), nullptr) != 0)
      H->submit_rst_stream(c->s, 0, call->stream, h2::INTERNAL_ERROR);
    else if (call->rejected)             // answered mid-request: stop the client's upload once the status is out
      c->rst_after.push_back(call->stream);
  }
}

void GrpcFront::Impl::slow_loop() {
  for (;;) {
    CallP call;
    {
      std::unique_lock<std::mutex> lk(qmu);
      qcv.wait(lk, [&] { return sstop || !sq.empty(); });
      if (sstop) return;
      call = std::move(sq.front());
      sq.pop_front();
    }
    SlowReply r;
    try {
      r = slow(call->path, call->body.substr(5), call->deadline_us);
    } catch (const std::exception& e) {
      r = SlowReply{};
      r.code = G_INTERNAL;
      r.message = e.what();
    }
    call->code = r.code;
    call->message = std::move(r.message);
    call->meta = std::move(r.meta);
    try {
      if (r.code == G_OK) call->resp = grpc_frame(r.body);
    } catch (const std::bad_alloc&) {
      set_error(*call, G_RESOURCE, "out of memory building the response");
    }
    std::string().swap(call->body);      // the request is no longer needed
    if (call->budget && call->held) call->budget->fetch_sub(call->held, std::memory_order_relaxed);
    call->held = 0;
    mail->post(call);
  }
}

// ---------------------------------------------------------------- connections
void GrpcFront::Impl::want_out(Worker* w, Conn* c, bool on) {
  if (c->pollout == on) return;
  c->pollout = on;
  epoll_event ev{};
  ev.events = on ? uint32_t(EPOLLIN | EPOLLOUT) : uint32_t(EPOLLIN);
  ev.data.u64 = c->id;
  epoll_ctl(w->ep, EPOLL_CTL_MOD, c->fd, &ev);
}

void GrpcFront::Impl::close_conn(Worker* w, Conn* c) {
  epoll_ctl(w->ep, EPOLL_CTL_DEL, c->fd, nullptr);
  ::close(c->fd);
  H->session_del(c->s);
  {
    std::lock_guard<std::mutex> lk(stmu);
    --st.open_connections;
  }
  w->conns.erase(c->id);                 // pending calls stay alive in their batcher callbacks
}

bool GrpcFront::Impl::flush(Worker* w, Conn* c) {
  while (c->out_off < c->out.size()) {
    const ssize_t n = ::send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
    if (n > 0) {
      c->out_off += size_t(n);
    } else if (n < 0 && errno == EINTR) {
      continue;
    } else if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      want_out(w, c, true);
      return true;
    } else {
      close_conn(w, c);
      return false;
    }
  }
  c->out.clear();
  c->out_off = 0;
  for (;;) {
    const uint8_t* d = nullptr;
    const ssize_t n = H->mem_send(c->s, &d);
    if (n < 0) {
      close_conn(w, c);
      return false;
    }
    if (n == 0) {
      if (c->rst_after.empty()) break;
      for (int32_t sid : c->rst_after) H->submit_rst_stream(c->s, 0, sid, h2::NO_ERROR);
      c->rst_after.clear();
      continue;
    }
    size_t off = 0;
    while (off < size_t(n)) {
      const ssize_t k = ::send(c->fd, d + off, size_t(n) - off, MSG_NOSIGNAL);
      if (k > 0) {
        off += size_t(k);
      } else if (k < 0 && errno == EINTR) {
        continue;
      } else if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        c->out.assign(reinterpret_cast<const char*>(d) + off, size_t(n) - off);   // nghttp2 reuses d
        want_out(w, c, true);
        return true;
      } else {
        close_conn(w, c);
        return false;
      }
    }
  }
  want_out(w, c, false);
  if (!H->want_read(c->s) && !H->want_write(c->s)) {
    close_conn(w, c);
    return false;
  }
  return true;
}

void GrpcFront::Impl::on_readable(Worker* w, Conn* c) {
  for (int i = 0; i < 16; ++i) {         // bounded: other connections of this worker get their turn
    const ssize_t n = ::read(c->fd, w->rbuf.data(), w->rbuf.size());
    if (n > 0) {
      const ssize_t rv = H->mem_recv(c->s, w->rbuf.data(), size_t(n));
      std::vector<CallP> local;
      local.swap(w->local);
      for (const auto& call : local) answer(w, call);
      if (rv < 0) {
        close_conn(w, c);
        return;
      }
      if (size_t(n) < w->rbuf.size()) break;
      continue;
    }
    if (n < 0 && errno == EINTR) continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    close_conn(w, c);                    // EOF or error
    return;
  }
  flush(w, c);
}

void GrpcFront::Impl::accept_all(Worker* w) {
  for (;;) {
    const int fd = accept4(w->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR) continue;
      return;                            // EAGAIN (drained) or a transient error
    }
    const int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    auto c = std::make_unique<Conn>();
    c->id = uint64_t(w->idx) << 48 | w->next++;
    c->fd = fd;
    c->w = w;
    if (H->server_new(&c->s, cbs, c.get()) != 0) {
      ::close(fd);
      continue;
    }
    const h2::settings_entry iv[] = {{h2::SETTINGS_MAX_CONCURRENT_STREAMS, 1024},
                                     {h2::SETTINGS_INITIAL_WINDOW_SIZE, uint32_t(kStreamWindow)},
                                     {h2::SETTINGS_MAX_FRAME_SIZE, uint32_t(kMaxFrame)}};
    H->submit_settings(c->s, 0, iv, 3);
    H->set_local_window_size(c->s, 0, 0, kConnWindow);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = c->id;
    if (epoll_ctl(w->ep, EPOLL_CTL_ADD, fd, &ev) != 0) {
      H->session_del(c->s);
      ::close(fd);
      continue;
    }
    Conn* cp = c.get();
    w->conns.emplace(c->id, std::move(c));
    {
      std::lock_guard<std::mutex> lk(stmu);
      ++st.connections;
      ++st.open_connections;
    }
    flush(w, cp);                        // our SETTINGS
  }
}

void GrpcFront::Impl::run(Worker* w) {
  epoll_event evs[128];
  Mailbox::Box& box = *mail->box[size_t(w->idx)];
  std::vector<CallP> done;
  std::unordered_set<uint64_t> touched;
  while (!stopping.load(std::memory_order_acquire)) {
    const int n = epoll_wait(w->ep, evs, 128, -1);
    if (n < 0) {
      if (errno == EINTR) continue;
      break;
    }
    for (int i = 0; i < n; ++i) {
      const uint64_t id = evs[i].data.u64;
      if (id == kListenTag) {
        accept_all(w);
      } else if (id == kWakeTag) {
        uint64_t v;
        (void)!::read(w->efd, &v, sizeof v);
        {
          std::lock_guard<std::mutex> lk(box.mu);
          done.swap(box.q);
        }
        touched.clear();
        for (const auto& call : done) {
          try {
            answer(w, call);
          } catch (...) {                  // e.g. bad_alloc building a response: reset that stream only
            auto ci = w->conns.find(call->conn);
            if (ci != w->conns.end()) H->submit_rst_stream(ci->second->s, 0, call->stream, h2::INTERNAL_ERROR);
          }
          touched.insert(call->conn);
        }
        done.clear();
        for (uint64_t cid : touched) {
          auto it = w->conns.find(cid);
          if (it != w->conns.end()) flush(w, it->second.get());
        }
      } else {
        auto it = w->conns.find(id);
        if (it == w->conns.end()) continue;
        try {
          if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) on_readable(w, it->second.get());
          else if (evs[i].events & EPOLLOUT) flush(w, it->second.get());
        } catch (...) {                    // outside the nghttp2 callbacks (answer, flush): drop the connection
          w->local.clear();
          auto again = w->conns.find(id);
          if (again != w->conns.end()) close_conn(w, again->second.get());
        }
      }
    }
  }
  while (!w->conns.empty()) close_conn(w, w->conns.begin()->second.get());
}

// ---------------------------------------------------------------- GrpcFront
GrpcFront::GrpcFront(const std::string& host, int port, int io_threads, int slow_threads, SlowFn slow,
                     size_t max_recv_bytes, bool reuse_port)
    : p_(std::make_unique<Impl>()) {
  std::string why;
  p_->H = h2::api(&why);
  if (!p_->H) throw std::runtime_error(why);
  if (io_threads < 1 || slow_threads < 1 || !slow) throw std::invalid_argument("GrpcFront: bad arguments");
  if (max_recv_bytes < 64 || max_recv_bytes > (size_t(1) << 31) - 1)
    throw std::invalid_argument("GrpcFront: max_recv_bytes out of range [64, 2^31)");
  Impl& I = *p_;
  I.slow = std::move(slow);
  I.max_recv = max_recv_bytes;
  I.max_held = std::max<int64_t>(int64_t(16) * int64_t(max_recv_bytes), int64_t(256) << 20);
  I.H->callbacks_new(&I.cbs);
  I.H->set_on_begin_headers(I.cbs, cb_begin_headers);
  I.H->set_on_header(I.cbs, cb_header);
  I.H->set_on_frame_recv(I.cbs, cb_frame_recv);
  I.H->set_on_data_chunk_recv(I.cbs, cb_data_chunk);
  I.H->set_on_stream_close(I.cbs, cb_stream_close);

  std::string h = host;
  if (h.size() > 2 && h.front() == '[' && h.back() == ']') h = h.substr(1, h.size() - 2);
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE;
  if (getaddrinfo(h.empty() ? nullptr : h.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("GrpcFront: cannot resolve " + host);
  sockaddr_storage addr{};
  std::memcpy(&addr, res->ai_addr, res->ai_addrlen);
  const socklen_t alen = res->ai_addrlen;
  const int family = res->ai_family;
  freeaddrinfo(res);

  auto fail = [&](const std::string& what) {
    const std::string e = what + ": " + std::strerror(errno);
    stop();
    throw std::runtime_error("GrpcFront: " + e);
  };
  // The workers' listeners share the port through SO_REUSEPORT. Unless the port is meant to be
  // shared with other processes (--procs children), a server already bound there must make
  // this one fail, not silently take part of its connections: probe with a plain bind first.
  if (!reuse_port && port != 0) {
    const int probe = ::socket(family, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (probe < 0) fail("socket");
    const int one = 1;
    setsockopt(probe, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    const int rc = ::bind(probe, reinterpret_cast<sockaddr*>(&addr), alen);
    const int err = errno;
    ::close(probe);
    if (rc != 0) {
      errno = err;
      fail("bind " + host + ":" + std::to_string(port));
    }
  }
  for (int i = 0; i < io_threads; ++i) {
    auto w = std::make_unique<Worker>();
    w->impl = p_.get();
    w->idx = i;
    auto box = std::make_unique<Mailbox::Box>();
    box->efd = w->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    I.mail->box.push_back(std::move(box));
    Worker* wp = w.get();
    I.workers.push_back(std::move(w));
    if (wp->efd < 0) fail("eventfd");
    wp->ep = epoll_create1(EPOLL_CLOEXEC);
    if (wp->ep < 0) fail("epoll_create1");
    wp->lfd = ::socket(family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (wp->lfd < 0) fail("socket");
    const int one = 1;
    setsockopt(wp->lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    // one listener per worker (the kernel spreads connections), and --procs processes share the port
    setsockopt(wp->lfd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    if (::bind(wp->lfd, reinterpret_cast<sockaddr*>(&addr), alen) != 0) fail("bind " + host + ":" + std::to_string(port));
    if (::listen(wp->lfd, 1024) != 0) fail("listen");
    if (i == 0) {                        // port 0: every further listener binds the chosen port
      sockaddr_storage got{};
      socklen_t gl = sizeof got;
      getsockname(wp->lfd, reinterpret_cast<sockaddr*>(&got), &gl);
      const uint16_t p = family == AF_INET6 ? reinterpret_cast<sockaddr_in6*>(&got)->sin6_port
                                            : reinterpret_cast<sockaddr_in*>(&got)->sin_port;
      if (family == AF_INET6) reinterpret_cast<sockaddr_in6*>(&addr)->sin6_port = p;
      else reinterpret_cast<sockaddr_in*>(&addr)->sin_port = p;
      I.port = ntohs(p);
    }
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = kListenTag;
    epoll_ctl(wp->ep, EPOLL_CTL_ADD, wp->lfd, &ev);
    ev.data.u64 = kWakeTag;
    epoll_ctl(wp->ep, EPOLL_CTL_ADD, wp->efd, &ev);
  }
  for (auto& w : I.workers) {
    Worker* wp = w.get();
    wp->th = std::thread([this, wp] { p_->run(wp); });
  }
  for (int i = 0; i < slow_threads; ++i) I.slow_threads.emplace_back([this] { p_->slow_loop(); });
}

GrpcFront::~GrpcFront() {
  stop();
  if (p_->cbs) p_->H->callbacks_del(p_->cbs);
}

int GrpcFront::port() const { return p_->port; }

void GrpcFront::set_route(FrontRoute r) {
  if (!r.batcher || r.image <= 0 || r.out_cols <= 0 || (r.dtype != 1 && r.dtype != 4))
    throw std::invalid_argument("GrpcFront::set_route: incomplete route");
  const std::string key = r.model + '\0' + r.signature;
  auto route = std::make_shared<const FrontRoute>(std::move(r));
  std::lock_guard<std::mutex> lk(p_->rmu);
  auto m = std::make_shared<Impl::RouteMap>(*p_->routes);
  (*m)[key] = std::move(route);
  p_->routes = std::move(m);
}

void GrpcFront::clear_routes() {
  std::lock_guard<std::mutex> lk(p_->rmu);
  p_->routes = std::make_shared<Impl::RouteMap>();
}

void GrpcFront::stop() {
  Impl& I = *p_;
  std::lock_guard<std::mutex> lk(I.stop_mu);
  if (I.stopped) return;
  I.stopped = true;
  I.stopping.store(true, std::memory_order_release);
  I.mail->closed.store(true, std::memory_order_release);
  for (auto& w : I.workers) {
    if (w->efd >= 0) {
      const uint64_t one = 1;
      (void)!::write(w->efd, &one, sizeof one);
    }
  }
  for (auto& w : I.workers) {
    if (w->th.joinable()) w->th.join();
    if (w->lfd >= 0) ::close(w->lfd);
    if (w->ep >= 0) ::close(w->ep);
    w->lfd = w->ep = -1;                 // the eventfd belongs to the mailbox
  }
  {
    std::lock_guard<std::mutex> q(I.qmu);
    I.sstop = true;
    I.sq.clear();
  }
  I.qcv.notify_all();
  for (auto& t : I.slow_threads)
    if (t.joinable()) t.join();
  clear_routes();
}

FrontStats GrpcFront::stats() const {
  std::lock_guard<std::mutex> lk(p_->stmu);
  return p_->st;
}

}  // namespace kdl
