// HTTP/2 framing for the native gRPC front-end (grpc_front.h) and its load generator: the
// system libnghttp2 (HPACK, framing, flow control), loaded with dlopen at first use so that
// kdl._rt imports on hosts without it (the front-end then reports unavailable and the server
// keeps the grpcio one). The image ships the library without headers, so the subset of its
// C API used here is declared below -- the public, ABI-stable nghttp2 1.x surface
// (struct layouts are part of that ABI: nghttp2_nv, nghttp2_frame_hd, nghttp2_data_provider,
// nghttp2_settings_entry).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>

#include <string>

namespace kdl::h2 {

struct session;                       // nghttp2_session (opaque)
struct callbacks;                     // nghttp2_session_callbacks (opaque)

struct nv {                           // nghttp2_nv
  uint8_t* name;
  uint8_t* value;
  size_t namelen, valuelen;
  uint8_t flags;
};
struct frame_hd {                     // nghttp2_frame_hd: first member of every nghttp2_frame
  size_t length;
  int32_t stream_id;
  uint8_t type, flags, reserved;
};
struct settings_entry {               // nghttp2_settings_entry
  int32_t settings_id;
  uint32_t value;
};
union data_source {                   // nghttp2_data_source
  int fd;
  void* ptr;
};
using read_cb = ssize_t (*)(session*, int32_t stream_id, uint8_t* buf, size_t length, uint32_t* data_flags,
                            data_source* source, void* user_data);
struct data_provider {                // nghttp2_data_provider
  data_source source;
  read_cb read_callback;
};

using begin_headers_cb = int (*)(session*, const frame_hd*, void*);
using header_cb = int (*)(session*, const frame_hd*, const uint8_t*, size_t, const uint8_t*, size_t, uint8_t, void*);
using frame_recv_cb = int (*)(session*, const frame_hd*, void*);
using data_chunk_cb = int (*)(session*, uint8_t flags, int32_t stream_id, const uint8_t*, size_t, void*);
using stream_close_cb = int (*)(session*, int32_t stream_id, uint32_t error_code, void*);

enum : uint8_t { FRAME_DATA = 0, FRAME_HEADERS = 1, FLAG_END_STREAM = 1 };
enum : uint32_t { DATA_FLAG_EOF = 1, DATA_FLAG_NO_END_STREAM = 2 };
enum : int32_t {
  SETTINGS_HEADER_TABLE_SIZE = 1, SETTINGS_MAX_CONCURRENT_STREAMS = 3, SETTINGS_INITIAL_WINDOW_SIZE = 4,
  SETTINGS_MAX_FRAME_SIZE = 5, SETTINGS_MAX_HEADER_LIST_SIZE = 6,
};
constexpr int ERR_DEFERRED = -508;            // NGHTTP2_ERR_DEFERRED (read callback: no data yet)
constexpr int ERR_CALLBACK_FAILURE = -902;    // NGHTTP2_ERR_CALLBACK_FAILURE
constexpr uint32_t NO_ERROR = 0;              // RST_STREAM / GOAWAY error codes
constexpr uint32_t INTERNAL_ERROR = 2;

// the loaded entry points (the frame-typed callbacks take nghttp2_frame*, whose first
// member is the frame header: declared here with frame_hd* -- the same pointer)
struct Api {
  int (*callbacks_new)(callbacks**);
  void (*callbacks_del)(callbacks*);
  void (*set_on_begin_headers)(callbacks*, begin_headers_cb);
  void (*set_on_header)(callbacks*, header_cb);
  void (*set_on_frame_recv)(callbacks*, frame_recv_cb);
  void (*set_on_data_chunk_recv)(callbacks*, data_chunk_cb);
  void (*set_on_stream_close)(callbacks*, stream_close_cb);
  int (*server_new)(session**, const callbacks*, void* user_data);
  int (*client_new)(session**, const callbacks*, void* user_data);
  void (*session_del)(session*);
  ssize_t (*mem_recv)(session*, const uint8_t* in, size_t inlen);
  ssize_t (*mem_send)(session*, const uint8_t** data);
  int (*want_read)(session*);
  int (*want_write)(session*);
  int (*set_local_window_size)(session*, uint8_t flags, int32_t stream_id, int32_t window_size);
  int (*submit_settings)(session*, uint8_t flags, const settings_entry* iv, size_t niv);
  int (*submit_response)(session*, int32_t stream_id, const nv* nva, size_t nvlen, const data_provider* data);
  int (*submit_trailer)(session*, int32_t stream_id, const nv* nva, size_t nvlen);
  int32_t (*submit_request)(session*, const void* pri_spec, const nv* nva, size_t nvlen, const data_provider* data,
                            void* stream_user_data);
  int (*submit_rst_stream)(session*, uint8_t flags, int32_t stream_id, uint32_t error_code);
  int (*submit_goaway)(session*, uint8_t flags, int32_t last_stream_id, uint32_t error_code, const uint8_t* opaque,
                       size_t opaque_len);
  int (*resume_data)(session*, int32_t stream_id);
};

// nullptr (and the reason in *why) when libnghttp2 cannot be loaded
const Api* api(std::string* why = nullptr);

inline nv make_nv(const std::string& n, const std::string& v) {
  return nv{(uint8_t*)n.data(), (uint8_t*)v.data(), n.size(), v.size(), 0};
}

}  // namespace kdl::h2
