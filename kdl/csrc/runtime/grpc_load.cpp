#include "grpc_load.h"

#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstring>
#include <mutex>
#include <string_view>
#include <thread>
#include <unordered_map>

#include "batcher.h"
#include "h2.h"

namespace kdl {

namespace {

struct Stream {
  int64_t t0 = 0;
  size_t off = 0;
  int status = -1;
};

struct Client {
  const h2::Api* H = nullptr;
  h2::session* s = nullptr;
  const std::string* req = nullptr;      // framed request
  std::unordered_map<int32_t, Stream> st;
  int inflight = 0;
  int64_t warm_us = 0;
  LoadResult r;
};

int cl_header(h2::session*, const h2::frame_hd* f, const uint8_t* n, size_t nl, const uint8_t* v, size_t vl, uint8_t,
              void* ud) {
  if (std::string_view(reinterpret_cast<const char*>(n), nl) != "grpc-status") return 0;
  auto* c = static_cast<Client*>(ud);
  auto it = c->st.find(f->stream_id);
  if (it != c->st.end()) it->second.status = std::atoi(std::string(reinterpret_cast<const char*>(v), vl).c_str());
  return 0;
}

int cl_data(h2::session*, uint8_t, int32_t, const uint8_t*, size_t, void*) { return 0; }

int cl_close(h2::session*, int32_t sid, uint32_t err, void* ud) {
  auto* c = static_cast<Client*>(ud);
  auto it = c->st.find(sid);
  if (it == c->st.end()) return 0;
  const int64_t now = now_us();
  if (it->second.t0 >= c->warm_us) {
    const int code = err ? -1 : it->second.status;
    ++c->r.codes[code];
    if (code == 0) {
      ++c->r.ok;
      c->r.lat_ms.push_back((now - it->second.t0) * 1e-3);
    } else {
      ++c->r.failed;
    }
  }
  c->st.erase(it);
  --c->inflight;
  return 0;
}

ssize_t cl_read(h2::session*, int32_t sid, uint8_t* buf, size_t len, uint32_t* flags, h2::data_source* src, void*) {
  auto* c = static_cast<Client*>(src->ptr);
  auto it = c->st.find(sid);
  if (it == c->st.end()) return h2::ERR_CALLBACK_FAILURE;
  const size_t n = std::min(len, c->req->size() - it->second.off);
  std::memcpy(buf, c->req->data() + it->second.off, n);
  it->second.off += n;
  if (it->second.off == c->req->size()) *flags |= h2::DATA_FLAG_EOF;
  return ssize_t(n);
}

bool send_all(int fd, const uint8_t* d, size_t n) {
  while (n) {
    const ssize_t k = ::send(fd, d, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    d += k;
    n -= size_t(k);
  }
  return true;
}

void one_connection(const h2::Api* H, const sockaddr_storage& addr, socklen_t alen, int family,
                    const std::string& authority, const std::string& path, const std::string& req, int streams,
                    int64_t warm_us, int64_t end_us, int64_t give_up_us, const std::string& timeout_hdr,
                    LoadResult* out, std::mutex* mu) {
  Client c;
  c.H = H;
  c.req = &req;
  c.warm_us = warm_us;
  const int fd = ::socket(family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  const int one = 1;
  auto finish = [&](const char* err) {
    if (c.s) H->session_del(c.s);
    if (fd >= 0) ::close(fd);
    std::lock_guard<std::mutex> lk(*mu);
    if (err && out->error.empty()) out->error = err;
    out->ok += c.r.ok;
    out->failed += c.r.failed;
    out->lat_ms.insert(out->lat_ms.end(), c.r.lat_ms.begin(), c.r.lat_ms.end());
    for (auto& kv : c.r.codes) out->codes[kv.first] += kv.second;
  };
  if (fd < 0 || ::connect(fd, reinterpret_cast<const sockaddr*>(&addr), alen) != 0) return finish("connect failed");
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  h2::callbacks* cbs = nullptr;
  H->callbacks_new(&cbs);
  H->set_on_header(cbs, cl_header);
  H->set_on_data_chunk_recv(cbs, cl_data);
  H->set_on_stream_close(cbs, cl_close);
  const int rc = H->client_new(&c.s, cbs, &c);
  H->callbacks_del(cbs);
  if (rc != 0) return finish("nghttp2 client session");
  const h2::settings_entry iv[] = {{h2::SETTINGS_INITIAL_WINDOW_SIZE, 8u << 20}};
  H->submit_settings(c.s, 0, iv, 1);
  static const std::string km = ":method", vm = "POST", ksch = ":scheme", vsch = "http", kp = ":path", ka = ":authority",
                           kct = "content-type", vct = "application/grpc", kte = "te", vte = "trailers",
                           kto = "grpc-timeout";
  const h2::nv nva[] = {h2::make_nv(km, vm),  h2::make_nv(ksch, vsch), h2::make_nv(kp, path),
                        h2::make_nv(ka, authority), h2::make_nv(kct, vct), h2::make_nv(kte, vte),
                        h2::make_nv(kto, timeout_hdr)};
  std::vector<uint8_t> buf(size_t(1) << 16);
  for (;;) {
    const int64_t now = now_us();
    if ((now >= end_us && c.inflight == 0) || now >= give_up_us) break;
    while (now < end_us && c.inflight < streams) {
      h2::data_provider dp;
      dp.source.ptr = &c;
      dp.read_callback = cl_read;
      const int32_t sid = H->submit_request(c.s, nullptr, nva, sizeof nva / sizeof nva[0], &dp, nullptr);
      if (sid < 0) return finish("submit_request failed");
      c.st[sid].t0 = now;
      ++c.inflight;
    }
    for (;;) {
      const uint8_t* d = nullptr;
      const ssize_t n = H->mem_send(c.s, &d);
      if (n < 0) return finish("nghttp2 send error");
      if (n == 0) break;
      if (!send_all(fd, d, size_t(n))) return finish("connection lost (send)");
    }
    pollfd p{fd, POLLIN, 0};
    if (::poll(&p, 1, 20) <= 0) continue;
    const ssize_t n = ::recv(fd, buf.data(), buf.size(), MSG_DONTWAIT);
    if (n == 0) return finish("connection closed by the server");
    if (n < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) continue;
      return finish("connection lost (recv)");
    }
    if (H->mem_recv(c.s, buf.data(), size_t(n)) < 0) return finish("nghttp2 protocol error");
  }
  finish(nullptr);
}

}  // namespace

LoadResult grpc_load(const std::string& host, int port, const std::string& path, const std::string& message,
                     int conns, int streams, double seconds, double warm_s, double timeout_s, bool raw_frame) {
  LoadResult out;
  std::string why;
  const h2::Api* H = h2::api(&why);
  if (!H) {
    out.error = why;
    return out;
  }
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
    out.error = "cannot resolve " + host;
    return out;
  }
  sockaddr_storage addr{};
  std::memcpy(&addr, res->ai_addr, res->ai_addrlen);
  const socklen_t alen = res->ai_addrlen;
  const int family = res->ai_family;
  freeaddrinfo(res);
  std::string req;
  if (raw_frame) {                       // the caller's bytes as they are (e.g. a length prefix that lies)
    req = message;
  } else {
    req.assign(5, '\0');
    const uint32_t n = uint32_t(message.size());
    req[1] = char(n >> 24), req[2] = char(n >> 16), req[3] = char(n >> 8), req[4] = char(n);
    req += message;
  }
  const int64_t t0 = now_us(), warm = t0 + int64_t(warm_s * 1e6), end = t0 + int64_t((warm_s + seconds) * 1e6);
  const int64_t give_up = end + int64_t(timeout_s * 1e6);
  const std::string authority = host + ":" + std::to_string(port);
  const std::string tmo = std::to_string(int64_t(timeout_s * 1000)) + "m";
  std::mutex mu;
  std::vector<std::thread> th;
  for (int i = 0; i < conns; ++i)
    th.emplace_back(one_connection, H, std::cref(addr), alen, family, std::cref(authority), std::cref(path),
                    std::cref(req), streams, warm, end, give_up, std::cref(tmo), &out, &mu);
  for (auto& t : th) t.join();
  out.seconds = seconds;
  return out;
}

}  // namespace kdl
