#include "tfproto.h"

#include <cstring>

namespace kdl {
namespace {

enum Wire { VARINT = 0, I64 = 1, LEN = 2, I32 = 5 };

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  const uint8_t* base;
  Reader(const uint8_t* b, size_t n, const uint8_t* root) : p(b), end(b + n), base(root) {}
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p >= end) throw ProtoError("truncated varint");
      const uint8_t b = *p++;
      v |= uint64_t(b & 0x7f) << shift;
      if (!(b & 0x80)) return v;
    }
    throw ProtoError("varint too long");
  }
  void tag(uint32_t* field, uint32_t* wire) {
    const uint64_t t = varint();
    *field = uint32_t(t >> 3);
    *wire = uint32_t(t & 7);
    if (*field == 0) throw ProtoError("field number 0");
  }
  Reader sub() {
    const uint64_t n = varint();
    if (n > uint64_t(end - p)) throw ProtoError("length past end of buffer");
    Reader r(p, size_t(n), base);
    p += n;
    return r;
  }
  std::string str() {
    Reader r = sub();
    return std::string(reinterpret_cast<const char*>(r.p), size_t(r.end - r.p));
  }
  void skip(uint32_t wire) {
    switch (wire) {
      case VARINT: varint(); break;
      case I64: if (end - p < 8) throw ProtoError("truncated fixed64"); p += 8; break;
      case LEN: sub(); break;
      case I32: if (end - p < 4) throw ProtoError("truncated fixed32"); p += 4; break;
      default: throw ProtoError("unsupported wire type " + std::to_string(wire));
    }
  }
  size_t offset() const { return size_t(p - base); }
};

void parse_shape(Reader r, TensorView* t) {
  uint32_t f, w;
  while (!r.done()) {
    r.tag(&f, &w);
    if (f == 2 && w == LEN) {
      Reader d = r.sub();
      int64_t size = 0;
      while (!d.done()) {
        uint32_t f2, w2;
        d.tag(&f2, &w2);
        if (f2 == 1 && w2 == VARINT) size = int64_t(d.varint());
        else d.skip(w2);
      }
      t->dims.push_back(size);
    } else if (f == 3 && w == VARINT) {
      t->unknown_rank = r.varint() != 0;
    } else {
      r.skip(w);
    }
  }
}

TensorView parse_tensor(Reader r) {
  TensorView t;
  uint32_t f, w;
  while (!r.done()) {
    r.tag(&f, &w);
    if (f == 1 && w == VARINT) {
      t.dtype = int(r.varint());
    } else if (f == 2 && w == LEN) {
      parse_shape(r.sub(), &t);
    } else if (f == 4 && w == LEN) {
      Reader c = r.sub();
      t.has_content = true;
      t.content_offset = size_t(c.p - c.base);
      t.content_size = size_t(c.end - c.p);
    } else if ((f == 5 || f == 6 || f == 7 || f == 10 || f == 11 || f == 13) && w == LEN) {
      // packed typed values: keep a view; the caller knows the element width
      Reader c = r.sub();
      if (!t.has_content) {
        t.values_field = int(f);
        t.content_offset = size_t(c.p - c.base);
        t.content_size = size_t(c.end - c.p);
      }
    } else if (f == 5 && w == I32) {           // unpacked float_val
      if (r.end - r.p < 4) throw ProtoError("truncated fixed32");
      t.values_field = 5;
      t.unpacked.insert(t.unpacked.end(), r.p, r.p + 4);
      r.p += 4;
    } else {
      r.skip(w);
    }
  }
  return t;
}

ModelSpecView parse_spec(Reader r) {
  ModelSpecView s;
  uint32_t f, w;
  while (!r.done()) {
    r.tag(&f, &w);
    if (f == 1 && w == LEN) s.name = r.str();
    else if (f == 3 && w == LEN) s.signature_name = r.str();
    else if (f == 4 && w == LEN) s.version_label = r.str();
    else if (f == 2 && w == LEN) {               // google.protobuf.Int64Value
      Reader v = r.sub();
      s.version = 0;
      while (!v.done()) {
        uint32_t f2, w2;
        v.tag(&f2, &w2);
        if (f2 == 1 && w2 == VARINT) s.version = int64_t(v.varint());
        else v.skip(w2);
      }
    } else {
      r.skip(w);
    }
  }
  return s;
}

// ---------------------------------------------------------------- writer
void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back(char(v | 0x80));
    v >>= 7;
  }
  o.push_back(char(v));
}
void put_tag(std::string& o, uint32_t field, uint32_t wire) { put_varint(o, (uint64_t(field) << 3) | wire); }
void put_len(std::string& o, uint32_t field, const std::string& payload) {
  put_tag(o, field, LEN);
  put_varint(o, payload.size());
  o += payload;
}

std::string spec_bytes(const ModelSpecView& s) {
  std::string o;
  if (!s.name.empty()) put_len(o, 1, s.name);
  if (s.version >= 0) {
    std::string v;
    if (s.version != 0) {
      put_tag(v, 1, VARINT);
      put_varint(v, uint64_t(s.version));
    }
    put_len(o, 2, v);
  }
  if (!s.signature_name.empty()) put_len(o, 3, s.signature_name);
  return o;
}

}  // namespace

PredictRequestView parse_predict_request(const uint8_t* data, size_t size) {
  PredictRequestView out;
  Reader r(data, size, data);
  uint32_t f, w;
  while (!r.done()) {
    r.tag(&f, &w);
    if (f == 1 && w == LEN) {
      out.spec = parse_spec(r.sub());
    } else if (f == 2 && w == LEN) {          // map<string, TensorProto> entry
      Reader e = r.sub();
      std::string key;
      TensorView t;
      bool have_val = false;
      while (!e.done()) {
        uint32_t f2, w2;
        e.tag(&f2, &w2);
        if (f2 == 1 && w2 == LEN) key = e.str();
        else if (f2 == 2 && w2 == LEN) { t = parse_tensor(e.sub()); have_val = true; }
        else e.skip(w2);
      }
      if (!have_val) t = TensorView();
      out.inputs.emplace_back(std::move(key), std::move(t));
    } else if (f == 3 && w == LEN) {
      out.output_filter.push_back(r.str());
    } else {
      r.skip(w);
    }
  }
  return out;
}

ModelSpecView parse_model_spec_request(const uint8_t* data, size_t size) {
  Reader r(data, size, data);
  uint32_t f, w;
  while (!r.done()) {
    r.tag(&f, &w);
    if (f == 1 && w == LEN) return parse_spec(r.sub());
    r.skip(w);
  }
  return ModelSpecView();
}

std::string build_predict_response(const std::vector<OutputTensor>& outputs, const ModelSpecView& spec) {
  std::string o;
  for (const auto& t : outputs) {
    std::string tp;
    put_tag(tp, 1, VARINT);
    put_varint(tp, 1);                         // DT_FLOAT
    std::string shape;
    int64_t n = 1;
    for (int64_t d : t.dims) {
      std::string dim;
      put_tag(dim, 1, VARINT);
      put_varint(dim, uint64_t(d));
      put_len(shape, 2, dim);
      n *= d;
    }
    put_len(tp, 2, shape);
    if (n > 0) {                               // packed float_val (field 5)
      put_tag(tp, 5, LEN);
      put_varint(tp, uint64_t(n) * 4);
      tp.append(reinterpret_cast<const char*>(t.values), size_t(n) * 4);
    }
    std::string entry;
    put_len(entry, 1, t.key);
    put_len(entry, 2, tp);
    put_len(o, 1, entry);
  }
  put_len(o, 2, spec_bytes(spec));
  return o;
}

}  // namespace kdl
