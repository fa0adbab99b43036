// h2.hpp -- the part of the nghttp2 C API (HTTP/2 framing + HPACK) that the
// native gRPC server and its load generator use.  The image ships the
// runtime library (libnghttp2.so.14, nghttp2 1.43) without its development
// headers, so the declarations are restated here from the library's public,
// stable C ABI (nghttp2/nghttp2.h of that release).  Only the frame header is
// read from nghttp2_frame (every frame type starts with it).
#pragma once

#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>

extern "C" {

typedef struct nghttp2_session nghttp2_session;
typedef struct nghttp2_session_callbacks nghttp2_session_callbacks;

typedef struct {
    size_t length;
    int32_t stream_id;
    uint8_t type;
    uint8_t flags;
    uint8_t reserved;
} nghttp2_frame_hd;

// every member of the nghttp2_frame union begins with the frame header
typedef union {
    nghttp2_frame_hd hd;
} nghttp2_frame;

typedef struct {
    uint8_t* name;
    uint8_t* value;
    size_t namelen;
    size_t valuelen;
    uint8_t flags;
} nghttp2_nv;

typedef struct {
    int32_t settings_id;
    uint32_t value;
} nghttp2_settings_entry;

typedef union {
    int fd;
    void* ptr;
} nghttp2_data_source;

typedef ssize_t (*nghttp2_data_source_read_callback)(nghttp2_session* session, int32_t stream_id, uint8_t* buf,
                                                     size_t length, uint32_t* data_flags,
                                                     nghttp2_data_source* source, void* user_data);
typedef struct {
    nghttp2_data_source source;
    nghttp2_data_source_read_callback read_callback;
} nghttp2_data_provider;

typedef int (*nghttp2_on_frame_recv_callback)(nghttp2_session* session, const nghttp2_frame* frame, void* user_data);
typedef int (*nghttp2_on_begin_headers_callback)(nghttp2_session* session, const nghttp2_frame* frame,
                                                 void* user_data);
typedef int (*nghttp2_on_header_callback)(nghttp2_session* session, const nghttp2_frame* frame, const uint8_t* name,
                                          size_t namelen, const uint8_t* value, size_t valuelen, uint8_t flags,
                                          void* user_data);
typedef int (*nghttp2_on_data_chunk_recv_callback)(nghttp2_session* session, uint8_t flags, int32_t stream_id,
                                                   const uint8_t* data, size_t len, void* user_data);
typedef int (*nghttp2_on_stream_close_callback)(nghttp2_session* session, int32_t stream_id, uint32_t error_code,
                                                void* user_data);

int nghttp2_session_callbacks_new(nghttp2_session_callbacks** callbacks_ptr);
void nghttp2_session_callbacks_del(nghttp2_session_callbacks* callbacks);
void nghttp2_session_callbacks_set_on_frame_recv_callback(nghttp2_session_callbacks* cbs,
                                                          nghttp2_on_frame_recv_callback cb);
void nghttp2_session_callbacks_set_on_begin_headers_callback(nghttp2_session_callbacks* cbs,
                                                             nghttp2_on_begin_headers_callback cb);
void nghttp2_session_callbacks_set_on_header_callback(nghttp2_session_callbacks* cbs, nghttp2_on_header_callback cb);
void nghttp2_session_callbacks_set_on_data_chunk_recv_callback(nghttp2_session_callbacks* cbs,
                                                               nghttp2_on_data_chunk_recv_callback cb);
void nghttp2_session_callbacks_set_on_stream_close_callback(nghttp2_session_callbacks* cbs,
                                                            nghttp2_on_stream_close_callback cb);

int nghttp2_session_server_new(nghttp2_session** session_ptr, const nghttp2_session_callbacks* callbacks,
                               void* user_data);
int nghttp2_session_client_new(nghttp2_session** session_ptr, const nghttp2_session_callbacks* callbacks,
                               void* user_data);
void nghttp2_session_del(nghttp2_session* session);
ssize_t nghttp2_session_mem_recv(nghttp2_session* session, const uint8_t* in, size_t inlen);
ssize_t nghttp2_session_mem_send(nghttp2_session* session, const uint8_t** data_ptr);
int nghttp2_session_want_read(nghttp2_session* session);
int nghttp2_session_want_write(nghttp2_session* session);
int nghttp2_submit_settings(nghttp2_session* session, uint8_t flags, const nghttp2_settings_entry* iv, size_t niv);
int nghttp2_submit_response(nghttp2_session* session, int32_t stream_id, const nghttp2_nv* nva, size_t nvlen,
                            const nghttp2_data_provider* data_prd);
int nghttp2_submit_trailer(nghttp2_session* session, int32_t stream_id, const nghttp2_nv* nva, size_t nvlen);
int32_t nghttp2_submit_request(nghttp2_session* session, const void* pri_spec, const nghttp2_nv* nva, size_t nvlen,
                               const nghttp2_data_provider* data_prd, void* stream_user_data);
int nghttp2_submit_goaway(nghttp2_session* session, uint8_t flags, int32_t last_stream_id, uint32_t error_code,
                          const uint8_t* opaque_data, size_t opaque_data_len);
int nghttp2_session_set_local_window_size(nghttp2_session* session, uint8_t flags, int32_t stream_id,
                                          int32_t window_size);
void* nghttp2_session_get_stream_user_data(nghttp2_session* session, int32_t stream_id);
int32_t nghttp2_session_get_last_proc_stream_id(nghttp2_session* session);

}  // extern "C"

namespace h2 {
// frame types / flags / settings ids / data flags (RFC 7540 and nghttp2.h)
constexpr uint8_t DATA = 0x0, HEADERS = 0x1;
constexpr uint8_t FLAG_END_STREAM = 0x1;
constexpr int32_t SETTINGS_MAX_CONCURRENT_STREAMS = 3, SETTINGS_INITIAL_WINDOW_SIZE = 4;
constexpr uint32_t DATA_FLAG_EOF = 0x1, DATA_FLAG_NO_END_STREAM = 0x2;
constexpr int ERR_CALLBACK_FAILURE = -902;

inline nghttp2_nv nv(const char* name, size_t nl, const char* value, size_t vl) {
    return nghttp2_nv{(uint8_t*)name, (uint8_t*)value, nl, vl, 0};
}
}  // namespace h2
