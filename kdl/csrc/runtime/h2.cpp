#include "h2.h"

#include <dlfcn.h>

#include <mutex>

namespace kdl::h2 {

namespace {

struct Loaded {
  Api api{};
  bool ok = false;
  std::string why;
};

template <class F>
bool sym(void* lib, const char* name, F& out, std::string& why) {
  out = reinterpret_cast<F>(dlsym(lib, name));
  if (!out && why.empty()) why = std::string("libnghttp2 lacks ") + name;
  return out != nullptr;
}

Loaded load() {
  Loaded L;
  void* lib = dlopen("libnghttp2.so.14", RTLD_NOW | RTLD_LOCAL);
  if (!lib) lib = dlopen("libnghttp2.so", RTLD_NOW | RTLD_LOCAL);
  if (!lib) {
    const char* e = dlerror();
    L.why = std::string("cannot load libnghttp2: ") + (e ? e : "?");
    return L;
  }
  Api& a = L.api;
  std::string& w = L.why;
  bool ok = sym(lib, "nghttp2_session_callbacks_new", a.callbacks_new, w);
  ok &= sym(lib, "nghttp2_session_callbacks_del", a.callbacks_del, w);
  ok &= sym(lib, "nghttp2_session_callbacks_set_on_begin_headers_callback", a.set_on_begin_headers, w);
  ok &= sym(lib, "nghttp2_session_callbacks_set_on_header_callback", a.set_on_header, w);
  ok &= sym(lib, "nghttp2_session_callbacks_set_on_frame_recv_callback", a.set_on_frame_recv, w);
  ok &= sym(lib, "nghttp2_session_callbacks_set_on_data_chunk_recv_callback", a.set_on_data_chunk_recv, w);
  ok &= sym(lib, "nghttp2_session_callbacks_set_on_stream_close_callback", a.set_on_stream_close, w);
  ok &= sym(lib, "nghttp2_session_server_new", a.server_new, w);
  ok &= sym(lib, "nghttp2_session_client_new", a.client_new, w);
  ok &= sym(lib, "nghttp2_session_del", a.session_del, w);
  ok &= sym(lib, "nghttp2_session_mem_recv", a.mem_recv, w);
  ok &= sym(lib, "nghttp2_session_mem_send", a.mem_send, w);
  ok &= sym(lib, "nghttp2_session_want_read", a.want_read, w);
  ok &= sym(lib, "nghttp2_session_want_write", a.want_write, w);
  ok &= sym(lib, "nghttp2_session_set_local_window_size", a.set_local_window_size, w);
  ok &= sym(lib, "nghttp2_submit_settings", a.submit_settings, w);
  ok &= sym(lib, "nghttp2_submit_response", a.submit_response, w);
  ok &= sym(lib, "nghttp2_submit_trailer", a.submit_trailer, w);
  ok &= sym(lib, "nghttp2_submit_request", a.submit_request, w);
  ok &= sym(lib, "nghttp2_submit_rst_stream", a.submit_rst_stream, w);
  ok &= sym(lib, "nghttp2_submit_goaway", a.submit_goaway, w);
  ok &= sym(lib, "nghttp2_session_resume_data", a.resume_data, w);
  L.ok = ok;                       // the library stays loaded for the process lifetime
  return L;
}

}  // namespace

const Api* api(std::string* why) {
  static const Loaded L = load();
  if (!L.ok && why) *why = L.why;
  return L.ok ? &L.api : nullptr;
}

}  // namespace kdl::h2
