/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see ref_ops.c).  CPU restatement of the reference's graph
 * walker and tensor plumbing:
 *   inference()            model_inference.rs:29-120 (nodes run in file order; the reference's
 *                          branch threads produce the same values, they only reorder siblings)
 *   node_inference()       model_inference.rs:128-162 (op_type dispatch, unknown op = error)
 *   get_stored_tensor()    utils.rs:113-185 (initializer decode on EVERY op call; shape from
 *                          graph.input, falling back to TensorProto.dims when not listed)
 *   manage_input_data()    utils.rs:29-45 (graph inputs that are not initializers are seeded)
 * Extensions, all documented in DESIGN.md: batch N (leading dim of the seeded input), the
 * Softmax result is stored in the value map (the reference only prints it, softmax_op.rs:30-41),
 * Reshape of an activation keeps the batch as the leading dim.
 * Errors replace the reference's panics: -1 plus a thread-local message.
 *
 * Minimal protobuf wire decoding, field numbers from /root/reference/models/onnx.proto.
 */
#define _GNU_SOURCE
#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ref_ops.h"

static _Thread_local char g_err[512];

static int fail(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return -1;
}

const char* oref_last_error(void) { return g_err; }

/* ------------------------------------------------------------------ protobuf wire decoding */
typedef struct { const uint8_t* p; int64_t n; } span_t;

static int rd_varint(const uint8_t** p, const uint8_t* end, uint64_t* out) {
  uint64_t r = 0;
  int shift = 0;
  while (*p < end) {
    uint8_t b = *(*p)++;
    r |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) { *out = r; return 0; }
    shift += 7;
    if (shift > 63) return -1;
  }
  return -1;
}

typedef struct { int fno, wt; uint64_t v; span_t s; } field_t;

static int next_field(const uint8_t** p, const uint8_t* end, field_t* f) {
  uint64_t key;
  if (rd_varint(p, end, &key)) return -1;
  f->fno = (int)(key >> 3);
  f->wt = (int)(key & 7);
  f->s.p = NULL; f->s.n = 0; f->v = 0;
  switch (f->wt) {
    case 0: return rd_varint(p, end, &f->v);
    case 1: if (end - *p < 8) return -1; f->s.p = *p; f->s.n = 8; *p += 8; return 0;
    case 5: if (end - *p < 4) return -1; f->s.p = *p; f->s.n = 4; *p += 4; return 0;
    case 2: {
      uint64_t ln;
      if (rd_varint(p, end, &ln) || (uint64_t)(end - *p) < ln) return -1;
      f->s.p = *p; f->s.n = (int64_t)ln; *p += ln; return 0;
    }
    default: return -1;
  }
}

static char* dup_span(span_t s) {
  char* r = (char*)malloc((size_t)s.n + 1);
  memcpy(r, s.p, (size_t)s.n);
  r[s.n] = 0;
  return r;
}

typedef struct { int64_t* v; int n, cap; } i64vec;
static void i64_push(i64vec* a, int64_t x) {
  if (a->n == a->cap) { a->cap = a->cap ? a->cap * 2 : 8; a->v = (int64_t*)realloc(a->v, (size_t)a->cap * 8); }
  a->v[a->n++] = x;
}
static void push_varints(i64vec* a, field_t* f) {
  if (f->wt == 0) { i64_push(a, (int64_t)f->v); return; }
  const uint8_t* p = f->s.p; const uint8_t* e = p + f->s.n; uint64_t v;
  while (p < e && !rd_varint(&p, e, &v)) i64_push(a, (int64_t)v);
}

typedef struct {
  char* name;
  i64vec dims;
  int dtype;
  span_t raw;          /* raw_data bytes (decoded on every get_stored_tensor call) */
  span_t fdata;        /* packed float_data bytes */
  float* fdata_unpacked; int n_fdata_unpacked;
  i64vec i64data;
} tproto;

typedef struct { char* name; int64_t i; float f; char* s; i64vec ints; } aproto;

typedef struct {
  char* op; char** in; int n_in; char** out; int n_out; aproto* at; int n_at;
} nproto;

typedef struct { char* name; i64vec shape; } vinfo;

struct oref_model {
  uint8_t* bytes; /* owned copy: initializer spans point into it */
  nproto* nodes; int n_nodes;
  tproto* inits; int n_inits;
  vinfo* inputs; int n_inputs;
  vinfo* outputs; int n_outputs;
  int64_t out_elems;
};

static void parse_tensor(span_t s, tproto* t) {
  memset(t, 0, sizeof *t);
  const uint8_t* p = s.p; const uint8_t* e = p + s.n; field_t f;
  while (p < e && !next_field(&p, e, &f)) {
    switch (f.fno) {
      case 1: push_varints(&t->dims, &f); break;
      case 2: t->dtype = (int)f.v; break;
      case 4:
        if (f.wt == 2) t->fdata = f.s;
        else if (f.wt == 5) {
          t->fdata_unpacked = (float*)realloc(t->fdata_unpacked, (size_t)(t->n_fdata_unpacked + 1) * 4);
          memcpy(&t->fdata_unpacked[t->n_fdata_unpacked++], f.s.p, 4);
        }
        break;
      case 7: push_varints(&t->i64data, &f); break;
      case 8: t->name = dup_span(f.s); break;
      case 9: t->raw = f.s; break;
      default: break;
    }
  }
  if (!t->name) t->name = strdup("");
}

static void parse_attr(span_t s, aproto* a) {
  memset(a, 0, sizeof *a);
  const uint8_t* p = s.p; const uint8_t* e = p + s.n; field_t f;
  while (p < e && !next_field(&p, e, &f)) {
    switch (f.fno) {
      case 1: a->name = dup_span(f.s); break;
      case 2: memcpy(&a->f, f.s.p, 4); break;
      case 3: a->i = (int64_t)f.v; break;
      case 4: a->s = dup_span(f.s); break;
      case 8: push_varints(&a->ints, &f); break;
      default: break;
    }
  }
  if (!a->name) a->name = strdup("");
}

static void parse_node(span_t s, nproto* n) {
  memset(n, 0, sizeof *n);
  const uint8_t* p = s.p; const uint8_t* e = p + s.n; field_t f;
  while (p < e && !next_field(&p, e, &f)) {
    if (f.fno == 1) { n->in = (char**)realloc(n->in, sizeof(char*) * (size_t)(n->n_in + 1)); n->in[n->n_in++] = dup_span(f.s); }
    else if (f.fno == 2) { n->out = (char**)realloc(n->out, sizeof(char*) * (size_t)(n->n_out + 1)); n->out[n->n_out++] = dup_span(f.s); }
    else if (f.fno == 4) n->op = dup_span(f.s);
    else if (f.fno == 5) { n->at = (aproto*)realloc(n->at, sizeof(aproto) * (size_t)(n->n_at + 1)); parse_attr(f.s, &n->at[n->n_at++]); }
  }
  if (!n->op) n->op = strdup("");
}

static void parse_vinfo(span_t s, vinfo* v) {
  memset(v, 0, sizeof *v);
  const uint8_t* p = s.p; const uint8_t* e = p + s.n; field_t f;
  while (p < e && !next_field(&p, e, &f)) {
    if (f.fno == 1) v->name = dup_span(f.s);
    else if (f.fno == 2) { /* TypeProto */
      const uint8_t* p2 = f.s.p; const uint8_t* e2 = p2 + f.s.n; field_t g;
      while (p2 < e2 && !next_field(&p2, e2, &g)) {
        if (g.fno != 1) continue; /* tensor_type */
        const uint8_t* p3 = g.s.p; const uint8_t* e3 = p3 + g.s.n; field_t h;
        while (p3 < e3 && !next_field(&p3, e3, &h)) {
          if (h.fno != 2) continue; /* shape */
          const uint8_t* p4 = h.s.p; const uint8_t* e4 = p4 + h.s.n; field_t d;
          while (p4 < e4 && !next_field(&p4, e4, &d)) {
            if (d.fno != 1) continue;
            int64_t dv = -1;
            const uint8_t* p5 = d.s.p; const uint8_t* e5 = p5 + d.s.n; field_t dd;
            while (p5 < e5 && !next_field(&p5, e5, &dd)) if (dd.fno == 1) dv = (int64_t)dd.v;
            i64_push(&v->shape, dv);
          }
        }
      }
    }
  }
  if (!v->name) v->name = strdup("");
}

oref_model* oref_model_load(const uint8_t* bytes, int64_t len) {
  oref_model* m = (oref_model*)calloc(1, sizeof *m);
  m->bytes = (uint8_t*)malloc((size_t)len);
  memcpy(m->bytes, bytes, (size_t)len);
  bytes = m->bytes;
  const uint8_t* p = bytes; const uint8_t* e = bytes + len; field_t f;
  span_t graph = {NULL, 0};
  while (p < e && !next_field(&p, e, &f)) if (f.fno == 7) graph = f.s;
  if (!graph.p) { fail("model has no graph"); free(m->bytes); free(m); return NULL; }
  p = graph.p; e = graph.p + graph.n;
  while (p < e && !next_field(&p, e, &f)) {
    if (f.fno == 1) { m->nodes = (nproto*)realloc(m->nodes, sizeof(nproto) * (size_t)(m->n_nodes + 1)); parse_node(f.s, &m->nodes[m->n_nodes++]); }
    else if (f.fno == 5) { m->inits = (tproto*)realloc(m->inits, sizeof(tproto) * (size_t)(m->n_inits + 1)); parse_tensor(f.s, &m->inits[m->n_inits++]); }
    else if (f.fno == 11) { m->inputs = (vinfo*)realloc(m->inputs, sizeof(vinfo) * (size_t)(m->n_inputs + 1)); parse_vinfo(f.s, &m->inputs[m->n_inputs++]); }
    else if (f.fno == 12) { m->outputs = (vinfo*)realloc(m->outputs, sizeof(vinfo) * (size_t)(m->n_outputs + 1)); parse_vinfo(f.s, &m->outputs[m->n_outputs++]); }
  }
  return m;
}

void oref_model_free(oref_model* m) {
  if (!m) return;
  for (int i = 0; i < m->n_nodes; ++i) {
    nproto* n = &m->nodes[i];
    for (int j = 0; j < n->n_in; ++j) free(n->in[j]);
    for (int j = 0; j < n->n_out; ++j) free(n->out[j]);
    for (int j = 0; j < n->n_at; ++j) { free(n->at[j].name); free(n->at[j].s); free(n->at[j].ints.v); }
    free(n->in); free(n->out); free(n->at); free(n->op);
  }
  for (int i = 0; i < m->n_inits; ++i) {
    free(m->inits[i].name); free(m->inits[i].dims.v); free(m->inits[i].i64data.v); free(m->inits[i].fdata_unpacked);
  }
  for (int i = 0; i < m->n_inputs; ++i) { free(m->inputs[i].name); free(m->inputs[i].shape.v); }
  for (int i = 0; i < m->n_outputs; ++i) { free(m->outputs[i].name); free(m->outputs[i].shape.v); }
  free(m->nodes); free(m->inits); free(m->inputs); free(m->outputs); free(m->bytes); free(m);
}

/* ------------------------------------------------------------------ value map + tensor decode */
typedef struct { int ndim; int64_t d[4]; float* data; int64_t* idata; } otensor;
static int64_t numel(const otensor* t) { int64_t n = 1; for (int i = 0; i < t->ndim; ++i) n *= t->d[i]; return n; }
static void ofree(otensor* t) { free(t->data); free(t->idata); t->data = NULL; t->idata = NULL; }

typedef struct { char* name; otensor t; } mapent;
typedef struct { mapent* e; int n; } vmap;

static otensor* map_get(vmap* m, const char* name) {
  for (int i = 0; i < m->n; ++i) if (!strcmp(m->e[i].name, name)) return &m->e[i].t;
  return NULL;
}
static void map_put(vmap* m, const char* name, otensor t) {
  otensor* old = map_get(m, name);
  if (old) { ofree(old); *old = t; return; }
  m->e = (mapent*)realloc(m->e, sizeof(mapent) * (size_t)(m->n + 1));
  m->e[m->n].name = strdup(name);
  m->e[m->n].t = t;
  m->n++;
}
static void map_free(vmap* m) {
  for (int i = 0; i < m->n; ++i) { free(m->e[i].name); ofree(&m->e[i].t); }
  free(m->e);
}
/* The reference deep-clones map inputs at every op entry (e.g. relu_op.rs:14-16). */
static otensor clone_t(const otensor* s) {
  otensor t = *s;
  int64_t n = numel(s);
  t.data = s->data ? (float*)malloc((size_t)n * 4) : NULL;
  if (t.data) memcpy(t.data, s->data, (size_t)n * 4);
  t.idata = NULL;
  return t;
}

static const tproto* find_init(oref_model* m, const char* name) {
  for (int i = 0; i < m->n_inits; ++i) if (!strcmp(m->inits[i].name, name)) return &m->inits[i];
  return NULL;
}
static const vinfo* find_input(oref_model* m, const char* name) {
  for (int i = 0; i < m->n_inputs; ++i) if (!strcmp(m->inputs[i].name, name)) return &m->inputs[i];
  return NULL;
}

/* get_stored_tensor (utils.rs:113-185): decode the initializer bytes on every call. */
static int get_stored(oref_model* m, const char* name, otensor* out) {
  const tproto* t = find_init(m, name);
  if (!t) return fail("initializer '%s' not found", name);
  const vinfo* vi = find_input(m, name);
  const i64vec* shp = vi ? &vi->shape : &t->dims;
  if (shp->n < 1 || shp->n > 4) return fail("unsupported rank %d for '%s'", shp->n, name);
  memset(out, 0, sizeof *out);
  out->ndim = shp->n;
  for (int i = 0; i < shp->n; ++i) out->d[i] = shp->v[i];
  int64_t n = numel(out);
  if (t->raw.n > 0 && t->dtype != 7) {
    if (t->raw.n != n * 4) return fail("initializer '%s' size mismatch", name);
    out->data = (float*)malloc((size_t)n * 4);
    for (int64_t i = 0; i < n; ++i) { float v; memcpy(&v, t->raw.p + 4 * i, 4); out->data[i] = v; } /* u8_to_f32 LE */
  } else if (t->fdata.n > 0 || t->n_fdata_unpacked > 0) {
    int64_t have = t->fdata.n ? t->fdata.n / 4 : t->n_fdata_unpacked;
    if (have != n) return fail("initializer '%s' size mismatch", name);
    out->data = (float*)malloc((size_t)n * 4);
    if (t->fdata.n) memcpy(out->data, t->fdata.p, (size_t)n * 4);
    else memcpy(out->data, t->fdata_unpacked, (size_t)n * 4);
  } else if (t->i64data.n > 0 || (t->raw.n > 0 && t->dtype == 7)) {
    out->idata = (int64_t*)malloc((size_t)n * 8);
    if (t->i64data.n) { if (t->i64data.n != n) return fail("size mismatch '%s'", name); memcpy(out->idata, t->i64data.v, (size_t)n * 8); }
    else memcpy(out->idata, t->raw.p, (size_t)n * 8);
  } else return fail("initializer '%s' has no data", name);
  return 0;
}


/* fetch an activation from the map (cloned) or an initializer */
static int fetch(oref_model* m, vmap* vm, const char* name, otensor* out) {
  otensor* t = map_get(vm, name);
  if (t) { *out = clone_t(t); return 0; }
  return get_stored(m, name, out);
}

/* ------------------------------------------------------------------ ops (node level) */
static int op_conv(oref_model* m, vmap* vm, const nproto* n, int faithful) {
  otensor x, w, b = {0};
  if (n->n_in < 2) return fail("Conv needs 2 inputs");
  if (fetch(m, vm, n->in[0], &x)) return -1;
  if (fetch(m, vm, n->in[1], &w)) { ofree(&x); return -1; }
  if (n->n_in > 2 && get_stored(m, n->in[2], &b)) { ofree(&x); ofree(&w); return -1; }
  int auto_pad = 3; int64_t group = 1; const aproto* pads = NULL; const aproto* strides = NULL;
  int rc = 0;
  for (int i = 0; i < n->n_at && !rc; ++i) {
    const aproto* a = &n->at[i];
    if (!strcmp(a->name, "auto_pad")) {
      const char* s = a->s ? a->s : "";
      if (!strcmp(s, "SAME_UPPER")) auto_pad = 1; else if (!strcmp(s, "SAME_LOWER")) auto_pad = 2;
      else if (!strcmp(s, "VALID")) auto_pad = 3; else if (!strcmp(s, "NOT_SET")) auto_pad = 0;
      else rc = fail("Convolution Auto Pad specified not found: %s", s);
    } else if (!strcmp(a->name, "dilations")) {
      for (int j = 0; j < a->ints.n; ++j) if (a->ints.v[j] != 1) rc = fail("Conv dilation>1 unsupported");
    } else if (!strcmp(a->name, "group")) group = a->i;
    else if (!strcmp(a->name, "kernel_shape")) {}
    else if (!strcmp(a->name, "pads")) pads = a;
    else if (!strcmp(a->name, "strides")) strides = a;
    else rc = fail("ATTRIBUTE NAME FOR CONVOLUTION NOT FOUND, %s", a->name);
  }
  if (!rc && pads && pads->ints.n >= 4)
    for (int j = 0; j < 4; ++j) if (pads->ints.v[j] > 0) auto_pad = 0; /* :169-173 */
  if (!rc && (!strides || strides->ints.n < 2)) rc = fail("Conv strides missing");
  if (!rc && (x.ndim != 4 || w.ndim != 4)) rc = fail("Conv expects 4-D input and weight");
  if (!rc && (group != 1 || x.d[1] != w.d[1])) rc = fail("Conv group/channel mismatch");
  if (!rc && b.data && (b.ndim != 1 || b.d[0] != w.d[0])) rc = fail("Bias array has the wrong shape");
  int64_t p[4], Ho, Wo;
  if (!rc && oref_resolve_window(auto_pad, pads ? pads->ints.v : NULL, pads ? pads->ints.n : 0, x.d[2], x.d[3],
                                 w.d[2], w.d[3], strides->ints.v[0], strides->ints.v[1], p, &Ho, &Wo))
    rc = fail("Conv window resolution failed");
  if (!rc) {
    otensor y = {4, {x.d[0], w.d[0], Ho, Wo}, NULL, NULL};
    y.data = (float*)malloc((size_t)numel(&y) * 4);
    if (oref_conv2d(x.data, x.d[0], x.d[1], x.d[2], x.d[3], w.data, w.d[0], w.d[2], w.d[3], b.data, p,
                    strides->ints.v[0], strides->ints.v[1], Ho, Wo, y.data, faithful)) {
      ofree(&y); rc = fail("conv2d shape mismatch");
    } else map_put(vm, n->out[0], y);
  }
  ofree(&x); ofree(&w); ofree(&b);
  return rc;
}

static int op_maxpool(oref_model* m, vmap* vm, const nproto* n, int faithful) {
  otensor x;
  if (fetch(m, vm, n->in[0], &x)) return -1;
  int auto_pad = 3, rc = 0; const aproto *pads = NULL, *strides = NULL, *ks = NULL;
  for (int i = 0; i < n->n_at && !rc; ++i) {
    const aproto* a = &n->at[i];
    if (!strcmp(a->name, "auto_pad")) {
      const char* s = a->s ? a->s : "";
      if (!strcmp(s, "SAME_UPPER")) auto_pad = 1; else if (!strcmp(s, "SAME_LOWER")) auto_pad = 2;
      else if (!strcmp(s, "VALID")) auto_pad = 3; else if (!strcmp(s, "NOTSET")) auto_pad = 0;
      else rc = fail("MaxPool Auto Pad specified not found: %s", s);
    } else if (!strcmp(a->name, "kernel_shape")) ks = a;
    else if (!strcmp(a->name, "pads")) pads = a;
    else if (!strcmp(a->name, "storage_order")) {}
    else if (!strcmp(a->name, "strides")) strides = a;
    else rc = fail("ATTRIBUTE NAME FOR MAX POOL NOT FOUND, %s", a->name);
  }
  if (!rc && (!ks || ks->ints.n < 2)) rc = fail("MaxPool kernel_shape missing");
  if (!rc && (!strides || strides->ints.n < 2)) rc = fail("MaxPool strides missing");
  if (!rc && x.ndim != 4) rc = fail("MaxPool expects 4-D input");
  int64_t p[4], Ho, Wo;
  if (!rc && oref_resolve_window(auto_pad, pads ? pads->ints.v : NULL, pads ? pads->ints.n : 0, x.d[2], x.d[3],
                                 ks->ints.v[0], ks->ints.v[1], strides->ints.v[0], strides->ints.v[1], p, &Ho, &Wo))
    rc = fail("MaxPool window resolution failed");
  if (!rc) {
    otensor y = {4, {x.d[0], x.d[1], Ho, Wo}, NULL, NULL};
    y.data = (float*)malloc((size_t)numel(&y) * 4);
    if (oref_maxpool2d(x.data, x.d[0], x.d[1], x.d[2], x.d[3], ks->ints.v[0], ks->ints.v[1], p,
                       strides->ints.v[0], strides->ints.v[1], Ho, Wo, y.data, faithful)) {
      ofree(&y); rc = fail("max_pool2d shape mismatch");
    } else map_put(vm, n->out[0], y);
  }
  ofree(&x);
  return rc;
}

static int op_add(oref_model* m, vmap* vm, const nproto* n) {
  otensor a, b;
  if (n->n_in < 2) return fail("Add needs 2 inputs");
  if (find_init(m, n->in[0])) { if (get_stored(m, n->in[0], &a)) return -1; }
  else { otensor* t = map_get(vm, n->in[0]); if (!t) return fail("Cannot retrieve input 1 for Add operation from hashmap input/output"); a = clone_t(t); }
  if (!find_init(m, n->in[1])) { ofree(&a); return fail("Cannot retrieve input 2 for Add operation"); }
  if (get_stored(m, n->in[1], &b)) { ofree(&a); return -1; }
  int rc = 0;
  if (!(a.ndim == 4 && b.ndim == 3) && !(a.ndim == 2 && b.ndim == 2)) rc = fail("Add: unsupported ranks %d+%d", a.ndim, b.ndim);
  if (!rc) {
    otensor y = a; y.data = (float*)malloc((size_t)numel(&a) * 4); y.idata = NULL;
    if (oref_add_bcast(a.data, a.d, a.ndim, b.data, b.d, b.ndim, y.data)) { ofree(&y); rc = fail("Add: shapes not broadcastable"); }
    else map_put(vm, n->out[0], y);
  }
  ofree(&a); ofree(&b);
  return rc;
}

static int op_unary4(vmap* vm, const nproto* n, otensor* x) {
  otensor* t = map_get(vm, n->in[0]);
  if (!t || t->ndim != 4) return fail("%s expects a 4-D activation '%s'", n->op, n->in[0]);
  *x = clone_t(t);
  return 0;
}

static int run_node(oref_model* m, vmap* vm, const nproto* n, int faithful) {
  const char* op = n->op;
  if (!strcmp(op, "Conv")) return op_conv(m, vm, n, faithful);
  if (!strcmp(op, "MaxPool")) return op_maxpool(m, vm, n, faithful);
  if (!strcmp(op, "Add")) return op_add(m, vm, n);
  if (!strcmp(op, "Relu")) {
    otensor x; if (op_unary4(vm, n, &x)) return -1;
    otensor y = x; y.data = (float*)malloc((size_t)numel(&x) * 4);
    oref_relu(x.data, numel(&x), y.data); ofree(&x); map_put(vm, n->out[0], y); return 0;
  }
  if (!strcmp(op, "Dropout")) {
    for (int i = 0; i < n->n_at; ++i) if (strcmp(n->at[i].name, "ratio")) return fail("ATTRIBUTE NAME FOR DROP OUT NOT FOUND, %s", n->at[i].name);
    otensor x; if (op_unary4(vm, n, &x)) return -1;
    map_put(vm, n->out[0], x); return 0; /* identity: training_mode=false (dropout_op.rs:66-71) */
  }
  if (!strcmp(op, "GlobalAveragePool")) {
    otensor x; if (op_unary4(vm, n, &x)) return -1;
    otensor y = {4, {x.d[0], x.d[1], 1, 1}, NULL, NULL};
    y.data = (float*)malloc((size_t)(x.d[0] * x.d[1]) * 4);
    oref_gap(x.data, x.d[0], x.d[1], x.d[2] * x.d[3], y.data); ofree(&x); map_put(vm, n->out[0], y); return 0;
  }
  if (!strcmp(op, "Softmax")) {
    otensor x; if (op_unary4(vm, n, &x)) return -1;
    int64_t D = x.d[1] * x.d[2] * x.d[3];
    otensor y = {2, {x.d[0], D, 0, 0}, NULL, NULL};
    y.data = (float*)malloc((size_t)numel(&x) * 4);
    oref_softmax_rows(x.data, x.d[0], D, y.data); ofree(&x); map_put(vm, n->out[0], y); return 0;
  }
  if (!strcmp(op, "Concat")) {
    int64_t axis = 1;
    for (int i = 0; i < n->n_at; ++i) { if (strcmp(n->at[i].name, "axis")) return fail("ATTRIBUTE NAME FOR CONCATENATE NOT FOUND, %s", n->at[i].name); axis = n->at[i].i; }
    if (n->n_in != 2) return fail("Concat expects exactly 2 inputs");
    otensor* a = map_get(vm, n->in[0]); otensor* b = map_get(vm, n->in[1]);
    if (!a || !b || a->ndim != 4 || b->ndim != 4) return fail("Concat expects two 4-D activations");
    otensor ca = clone_t(a), cb = clone_t(b);
    otensor y = ca; y.idata = NULL;
    if (axis < 0 || axis > 3) { ofree(&ca); ofree(&cb); return fail("Concat axis out of range"); }
    y.d[axis] = ca.d[axis] + cb.d[axis];
    y.data = (float*)malloc((size_t)numel(&y) * 4);
    int rc = oref_concat2(ca.data, ca.d, cb.data, cb.d, (int)axis, y.data);
    ofree(&ca); ofree(&cb);
    if (rc) { ofree(&y); return fail("Concat shapes mismatch"); }
    map_put(vm, n->out[0], y); return 0;
  }
  if (!strcmp(op, "Reshape")) {
    otensor x, s;
    int from_init = find_init(m, n->in[0]) != NULL;
    if (from_init) { if (get_stored(m, n->in[0], &x)) return -1; }
    else { otensor* t = map_get(vm, n->in[0]); if (!t) return fail("Reshape input missing"); x = clone_t(t); }
    if (x.ndim != 4) { ofree(&x); return fail("Reshape expects 4-D data"); }
    if (!find_init(m, n->in[1])) { ofree(&x); return fail("Unable to retrieve Shape for Reshape operation"); }
    if (get_stored(m, n->in[1], &s) || !s.idata || s.ndim != 1 || s.d[0] < 2) { ofree(&x); ofree(&s); return fail("Reshape shape must be int64 [2]"); }
    int64_t ns[2] = {s.idata[0], s.idata[1]};
    for (int i = 0; i < 2; ++i) if (ns[i] == 0) ns[i] = x.d[i]; /* allowzero = 0 (:69-83) */
    ofree(&s);
    int64_t total = numel(&x);
    if (ns[0] < 0 || ns[1] < 0) { ofree(&x); return fail("Reshape: negative dims unsupported"); }
    if (ns[0] * ns[1] != total) {
      /* batch extension: a per-image shape [1, D] applied to N images -> [N, D] */
      if (!from_init && ns[0] == 1 && ns[1] * x.d[0] == total) ns[0] = x.d[0];
      else { ofree(&x); return fail("Reshape: element count mismatch"); }
    }
    otensor y = {2, {ns[0], ns[1], 0, 0}, x.data, NULL};
    map_put(vm, n->out[0], y); return 0;
  }
  if (!strcmp(op, "MatMul")) {
    otensor* a = map_get(vm, n->in[0]); otensor* b = map_get(vm, n->in[1]);
    if (!a || !b || a->ndim != 2 || b->ndim != 2 || a->d[1] != b->d[0]) return fail("MatMul expects two 2-D map tensors");
    otensor ca = clone_t(a), cb = clone_t(b);
    otensor y = {2, {ca.d[0], cb.d[1], 0, 0}, NULL, NULL};
    y.data = (float*)malloc((size_t)numel(&y) * 4);
    oref_matmul(ca.data, cb.data, ca.d[0], ca.d[1], cb.d[1], y.data);
    ofree(&ca); ofree(&cb); map_put(vm, n->out[0], y); return 0;
  }
  return fail("INFERENCE OPERATION '%s' NOT FOUND", op);
}

int oref_model_run(oref_model* m, const float* input, int64_t n, float* out, int64_t out_cap, int faithful) {
  vmap vm = {NULL, 0};
  int seeded = 0;
  for (int i = 0; i < m->n_inputs; ++i) {
    const vinfo* vi = &m->inputs[i];
    if (find_init(m, vi->name)) continue; /* manage_input_data skips initializers (utils.rs:35) */
    if (seeded) { map_free(&vm); return fail("oracle supports one seeded model input"); }
    if (vi->shape.n != 4) { map_free(&vm); return fail("model input must be 4-D"); }
    otensor t = {4, {n, vi->shape.v[1], vi->shape.v[2], vi->shape.v[3]}, NULL, NULL};
    t.data = (float*)malloc((size_t)numel(&t) * 4);
    memcpy(t.data, input, (size_t)numel(&t) * 4);
    map_put(&vm, vi->name, t);
    seeded = 1;
  }
  for (int i = 0; i < m->n_nodes; ++i)
    if (run_node(m, &vm, &m->nodes[i], faithful)) { map_free(&vm); return -1; }
  if (m->n_outputs < 1) { map_free(&vm); return fail("model has no outputs"); }
  otensor* y = map_get(&vm, m->outputs[0].name);
  if (!y) { map_free(&vm); return fail("graph output '%s' not produced", m->outputs[0].name); }
  int64_t ne = numel(y);
  m->out_elems = ne / n;
  if (ne > out_cap) { map_free(&vm); return fail("output buffer too small"); }
  memcpy(out, y->data, (size_t)ne * 4);
  map_free(&vm);
  return 0;
}

int64_t oref_model_out_elems(oref_model* m) { return m->out_elems; }
