// ONNX ModelProto loader (protobuf wire format, no libprotobuf in the image).
// Replaces the reference's `ModelProto::parse_from_bytes` (onnx-protobuf 0.2.3, main.rs:30)
// and the initializer decode of `get_stored_tensor` (utils.rs:113-185): initializers are
// decoded ONCE here (raw_data little-endian f32 / int64 by data_type, float_data,
// int64_data) instead of on every op call.  Field numbers: /root/reference/models/onnx.proto.
#include <cstring>

#include "ore_internal.h"

namespace ore {
namespace {

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;

  bool more() const { return ok && p < end; }
  uint64_t varint() {
    uint64_t r = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p >= end) { ok = false; return 0; }
      uint8_t b = *p++;
      r |= uint64_t(b & 0x7f) << shift;
      if (!(b & 0x80)) return r;
    }
    ok = false;
    return 0;
  }
  // One field: number, wire type, varint value or a [begin, end) payload.
  // Every out-parameter is written on every call (b / e are null for a varint), so a caller that
  // checks the wire type first never reads a stale or uninitialised payload pointer.
  bool next(int* fno, int* wt, uint64_t* v, const uint8_t** b, const uint8_t** e) {
    *v = 0;
    *b = *e = nullptr;
    uint64_t key = varint();
    if (!ok) return false;
    *fno = int(key >> 3);
    *wt = int(key & 7);
    switch (*wt) {
      case 0: *v = varint(); return ok;
      case 1: if (end - p < 8) return ok = false; *b = p; p += 8; *e = p; return true;
      case 5: if (end - p < 4) return ok = false; *b = p; p += 4; *e = p; return true;
      case 2: {
        uint64_t n = varint();
        if (!ok || uint64_t(end - p) < n) return ok = false;
        *b = p; p += n; *e = p; return true;
      }
      default: return ok = false;
    }
  }
};

// Wire-type contract of the fields this loader reads (onnx.proto): strings, bytes, sub-messages and
// packed repeated fields are length-delimited (2); scalar ints are varints (0); AttributeProto.f is
// a fixed32 (5).  A field whose wire type does not match is malformed input -> ORE_ERR_PARSE.
enum { WT_VARINT = 0, WT_FIXED64 = 1, WT_LEN = 2, WT_FIXED32 = 5 };

std::string str(const uint8_t* b, const uint8_t* e) { return std::string(reinterpret_cast<const char*>(b), e - b); }

bool packed_varints(int wt, uint64_t v, const uint8_t* b, const uint8_t* e, std::vector<int64_t>* out) {
  if (wt == WT_VARINT) { out->push_back(int64_t(v)); return true; }
  if (wt != WT_LEN) return false;
  Reader r{b, e};
  while (r.more()) out->push_back(int64_t(r.varint()));
  return r.ok;
}

// repeated float: packed (2, a whole number of 4-byte floats) or one unpacked fixed32 (5)
bool packed_floats(int wt, const uint8_t* b, const uint8_t* e, std::vector<float>* out) {
  if (wt != WT_LEN && wt != WT_FIXED32) return false;
  const size_t len = size_t(e - b);
  if (len % 4 != 0) return false;
  const size_t n = len / 4, off = out->size();
  out->resize(off + n);
  if (n) std::memcpy(out->data() + off, b, n * 4);
  return true;
}

bool parse_tensor(const uint8_t* b0, const uint8_t* e0, Initializer* t) {
  Reader r{b0, e0};
  const uint8_t *raw_b = nullptr, *raw_e = nullptr;
  int fno, wt; uint64_t v; const uint8_t *b, *e;
  while (r.more() && r.next(&fno, &wt, &v, &b, &e)) {
    bool ok = true;
    switch (fno) {
      case 1: ok = packed_varints(wt, v, b, e, &t->dims); break;
      case 2: ok = wt == WT_VARINT; t->dtype = int(v); break;
      case 4: ok = packed_floats(wt, b, e, &t->f32); break;
      case 7: ok = packed_varints(wt, v, b, e, &t->i64); break;
      case 8: ok = wt == WT_LEN; if (ok) t->name = str(b, e); break;
      case 9: ok = wt == WT_LEN; raw_b = b; raw_e = e; break;
      default: break;
    }
    if (!ok) return false;
  }
  if (!r.ok) return false;
  if (raw_b && raw_e > raw_b) {
    size_t n = size_t(raw_e - raw_b);
    if (t->dtype == 7) {  // INT64
      t->i64.resize(n / 8);
      std::memcpy(t->i64.data(), raw_b, (n / 8) * 8);
    } else {              // FLOAT (u8_to_f32: little-endian f32, utils.rs:192-197)
      t->f32.resize(n / 4);
      std::memcpy(t->f32.data(), raw_b, (n / 4) * 4);
    }
  }
  return true;
}

bool parse_attr(const uint8_t* b0, const uint8_t* e0, Attr* a) {
  Reader r{b0, e0};
  int fno, wt; uint64_t v; const uint8_t *b, *e;
  while (r.more() && r.next(&fno, &wt, &v, &b, &e)) {
    bool ok = true;
    switch (fno) {
      case 1: ok = wt == WT_LEN; if (ok) a->name = str(b, e); break;
      case 20: ok = wt == WT_VARINT; a->type = int(v); break;
      case 2:
        ok = wt == WT_FIXED32 && e - b == 4;
        if (ok) { std::memcpy(&a->f, b, 4); a->has_f = true; }
        break;
      case 3: ok = wt == WT_VARINT; a->i = int64_t(v); a->has_i = true; break;
      case 4: ok = wt == WT_LEN; if (ok) { a->s = str(b, e); a->has_s = true; } break;
      case 7: ok = packed_floats(wt, b, e, &a->floats); break;
      case 8: ok = packed_varints(wt, v, b, e, &a->ints); break;
      default: break;
    }
    if (!ok) return false;
  }
  return r.ok;
}

bool parse_node(const uint8_t* b0, const uint8_t* e0, Node* n) {
  Reader r{b0, e0};
  int fno, wt; uint64_t v; const uint8_t *b, *e;
  while (r.more() && r.next(&fno, &wt, &v, &b, &e)) {
    if (fno >= 1 && fno <= 5 && wt != WT_LEN) return false;
    switch (fno) {
      case 1: n->inputs.push_back(str(b, e)); break;
      case 2: n->outputs.push_back(str(b, e)); break;
      case 3: n->name = str(b, e); break;
      case 4: n->op_type = str(b, e); break;
      case 5: { n->attrs.emplace_back(); if (!parse_attr(b, e, &n->attrs.back())) return false; break; }
      default: break;
    }
  }
  return r.ok;
}

// ValueInfoProto -> name + TypeProto.tensor_type.shape dims (dim_param -> -1)
bool parse_value_info(const uint8_t* b0, const uint8_t* e0, ValueInfo* vi) {
  Reader r{b0, e0};
  int fno, wt; uint64_t v; const uint8_t *b, *e;
  while (r.more() && r.next(&fno, &wt, &v, &b, &e)) {
    if ((fno == 1 || fno == 2) && wt != WT_LEN) return false;
    if (fno == 1) { vi->name = str(b, e); continue; }
    if (fno != 2) continue;
    Reader t{b, e};
    int f2, w2; uint64_t v2; const uint8_t *b2, *e2;
    while (t.more() && t.next(&f2, &w2, &v2, &b2, &e2)) {
      if (f2 != 1) continue;  // tensor_type
      if (w2 != WT_LEN) return false;
      Reader tt{b2, e2};
      int f3, w3; uint64_t v3; const uint8_t *b3, *e3;
      while (tt.more() && tt.next(&f3, &w3, &v3, &b3, &e3)) {
        if (f3 != 2) continue;  // shape
        if (w3 != WT_LEN) return false;
        Reader sh{b3, e3};
        int f4, w4; uint64_t v4; const uint8_t *b4, *e4;
        while (sh.more() && sh.next(&f4, &w4, &v4, &b4, &e4)) {
          if (f4 != 1) continue;  // dim
          if (w4 != WT_LEN) return false;
          int64_t d = -1;
          Reader dm{b4, e4};
          int f5, w5; uint64_t v5; const uint8_t *b5, *e5;
          while (dm.more() && dm.next(&f5, &w5, &v5, &b5, &e5)) {
            if (f5 != 1) continue;  // dim_value (dim_param, 2, leaves -1)
            if (w5 != WT_VARINT) return false;
            d = int64_t(v5);
          }
          if (!dm.ok) return false;
          vi->shape.push_back(d);
        }
        if (!sh.ok) return false;
      }
      if (!tt.ok) return false;
    }
    if (!t.ok) return false;
  }
  return r.ok;
}

}  // namespace

bool parse_model(const uint8_t* data, size_t len, Graph* g, std::string* err) {
  Reader r{data, data + len};
  const uint8_t *gb = nullptr, *ge = nullptr;
  int fno, wt; uint64_t v; const uint8_t *b, *e;
  while (r.more() && r.next(&fno, &wt, &v, &b, &e))
    if (fno == 7) {
      if (wt != WT_LEN) { *err = "malformed ModelProto: graph is not length-delimited"; return false; }
      gb = b; ge = e;
    }
  if (!r.ok) { *err = "malformed ModelProto"; return false; }
  if (!gb) { *err = "ModelProto has no graph"; return false; }
  Reader gr{gb, ge};
  while (gr.more() && gr.next(&fno, &wt, &v, &b, &e)) {
    bool ok = true;
    if ((fno == 1 || fno == 5 || fno == 11 || fno == 12) && wt != WT_LEN) ok = false;
    else switch (fno) {
      case 1: g->nodes.emplace_back(); ok = parse_node(b, e, &g->nodes.back()); break;
      case 5: g->inits.emplace_back(); ok = parse_tensor(b, e, &g->inits.back()); break;
      case 11: g->inputs.emplace_back(); ok = parse_value_info(b, e, &g->inputs.back()); break;
      case 12: g->outputs.emplace_back(); ok = parse_value_info(b, e, &g->outputs.back()); break;
      default: break;
    }
    if (!ok) { *err = "malformed GraphProto field " + std::to_string(fno); return false; }
  }
  if (!gr.ok) { *err = "malformed GraphProto"; return false; }
  return true;
}

}  // namespace ore
