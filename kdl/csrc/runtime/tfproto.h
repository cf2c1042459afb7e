// Zero-copy TF-Serving PredictRequest parser and PredictResponse builder.
//
// TF-Serving decodes PredictRequest with the full protobuf runtime and copies
// every TensorProto into a Tensor. Here the raw gRPC bytes
// are walked once: each input's tensor_content is returned as an (offset, size)
// view into the request buffer, so a 1 MB f32 image goes straight from the
// gRPC receive buffer into the batcher's pinned staging slot with one memcpy.
// Responses are written with the typed float_val field, which is what the
// reference gateway reads (model_server.py:47).
#pragma once
#include <stdint.h>

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace kdl {

struct ProtoError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct TensorView {
  int dtype = 0;
  std::vector<int64_t> dims;
  bool unknown_rank = false;
  // tensor_content (or packed typed values) as a view into the request buffer
  size_t content_offset = 0, content_size = 0;
  bool has_content = false;
  int values_field = 0;                 // field number of packed *_val data when !has_content
  std::vector<uint8_t> unpacked;        // typed values that arrived unpacked (rare), as raw LE bytes
};

struct ModelSpecView {
  std::string name, signature_name, version_label;
  int64_t version = -1;                 // -1: not set
};

struct PredictRequestView {
  ModelSpecView spec;
  std::vector<std::pair<std::string, TensorView>> inputs;
  std::vector<std::string> output_filter;
};

PredictRequestView parse_predict_request(const uint8_t* data, size_t size);
ModelSpecView parse_model_spec_request(const uint8_t* data, size_t size);  // field 1 = ModelSpec

struct OutputTensor {
  std::string key;
  std::vector<int64_t> dims;
  const float* values;                  // row-major, prod(dims) floats
};
std::string build_predict_response(const std::vector<OutputTensor>& outputs, const ModelSpecView& spec);

}  // namespace kdl
