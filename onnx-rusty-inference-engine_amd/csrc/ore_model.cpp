// Graph walker: the device-resident replacement of `inference()` / `node_inference()`
// (model_inference.rs:29-162) and of the value map they share
// (`Arc<Mutex<HashMap<String, (Option<Array2>, Option<Array4>)>>>`, :30-32).
//
//  * Load: parse the ModelProto, upload every f32 initializer to HBM once (the reference
//    re-decodes them on every op call, utils.rs:113-185), run the reference's per-op shape and
//    attribute rules over the nodes in file order (the order the reference executes them in,
//    :84-115; its branch threads only reorder independent siblings), and turn each node into
//    a kernel step.  Anything the reference would panic on is reported here.
//  * Fuse (ORE_FUSE_*): Conv -> Relu into the conv epilogue; Concat(axis 1) of two
//    conv/pool outputs by writing both producers into channel slices of the concat buffer;
//    Dropout and activation Reshape as aliases.
//  * Plan: every materialised activation gets a slot in one device arena sized for max_batch,
//    slots reused by liveness (first-fit over [first write, last read] intervals).
//  * Run: launch the steps in order on the context stream; the model input and output are the
//    caller's device buffers.
//
// Batch: every activation carries a leading batch dim n (the reference is batch-1: it writes
// only image 0, e.g. convolution_op.rs:480).  Constants (initializers, Reshape of an
// initializer) carry none.
#include <algorithm>
#include <cstring>

#include "ore_internal.h"

using namespace ore;

namespace {

enum StepKind { S_CONV, S_MAXPOOL, S_RELU, S_ADD, S_SOFTMAX, S_MATMUL, S_GAP, S_CONCAT, S_COPY, S_NOP, S_FIRE };

struct Value {
  std::string name;
  bool is_const = false;
  bool is_input = false;
  bool is_output = false;
  int ndim = 0;
  int64_t dims[4] = {0, 0, 0, 0};  // activations: dims[0] = 1 (per image)
  float* cptr = nullptr;           // const f32 device data
  std::vector<int64_t> i64;        // const int64 host data
  bool has_i64 = false;
  int alias_of = -1;               // view into another value's storage
  int64_t alias_ch = 0;            // concat slice: first channel inside the base
  bool slice = false;              // alias is a channel slice of its base (Concat in place)
  int64_t ps = 0;                  // 4-D activations: channel-plane stride (>= H*W; padded planes),
                                   // or for nhwc values the pixel stride (the root's channel count)
  int es = 4;                      // element bytes: 4 f32, 2 f16 (f16 models, ORE_LOAD_F16)
  bool nhwc = false;               // channels-last storage (every 4-D f16 activation)
  bool elided = false;             // produced and consumed inside one fused kernel
  int64_t arena_off = -1;          // byte offset in the arena (root values)
  int first = -1, last = -1;       // live interval in step indices
  int uses = 0;                    // consumer count (node inputs)

  // elements between images in this value's own storage (roots)
  int64_t image_stride() const {
    if (ndim != 4 || !ps) return per_image();
    return nhwc ? dims[2] * dims[3] * ps : dims[1] * ps;
  }
  int64_t per_image() const {
    int64_t s = 1;
    for (int i = 1; i < ndim; ++i) s *= dims[i];
    return s;
  }
  int64_t numel_const() const {
    int64_t s = 1;
    for (int i = 0; i < ndim; ++i) s *= dims[i];
    return s;
  }
};

struct Step {
  StepKind kind = S_NOP;
  std::string op, name;
  int in0 = -1, in1 = -1, in2 = -1, out = -1;
  int in3 = -1;  // a fourth activation input: the recomputed expand1x1's input S (pe1)
  // conv / pool geometry (per image)
  int64_t C = 0, H = 0, W = 0, M = 0, kh = 0, kw = 0, sh = 1, sw = 1;
  Window win;
  bool relu = false;
  bool w_kmajor = false;  // MatMul: the constant operand is [K][M]
  // fused preceding MaxPool (pass pool_squeeze, pool_conv1x1_f32_kernel): in0 is the pool's input
  bool pool = false;
  int64_t pH = 0, pW = 0, psh = 1, psw = 1;
  Window pwin;
  // ... whose input is Concat(e1, e3) with e1 (a 1x1 conv + Relu of in3) recomputed inside the kernel
  // (pass pool_expand, ORE_FUSE_POOL_EXPAND): e1's K-major packing, its bias and shape
  bool pe1 = false;
  const float* pe1_w = nullptr;
  const float* pe1_b = nullptr;
  int64_t pe1_C = 0, pe1_E = 0;
  int pe1_Mp = 0;
  // fused following MaxPool (ORE_FUSE_CONV_POOL): out is the pool's output; pool geometry below
  bool epool = false;
  mutable int ran_tile = -1;  // pooled conv: the kernel variant its last launch took (EPOOL_TILE_BASE + v)
  int64_t ep_kh = 0, ep_kw = 0, ep_sh = 1, ep_sw = 1;
  Window ep_win;
  // S_FIRE (ORE_FUSE_FIRE): this squeeze conv also computes the fire module feeding it; in0 is the
  // fire's input S (C = its channels for the expands, fire_K = the squeeze's K = E1 + E3)
  int64_t fire_C = 0, fire_E1 = 0, fire_E3 = 0;
  const float* fire_w1 = nullptr;  // launch_fire_pack layouts of the expand weights
  const float* fire_w3 = nullptr;
  const float* fire_b1 = nullptr;
  const float* fire_b3 = nullptr;
  bool fire_f16 = false;           // f16 model: fire_f16_kernel, fire_w1 / fire_w3 / fire_ws16 in launch_fire_pack_f16 layout
  const void* fire_ws16 = nullptr;
  bool fire_pool = false;          // a 3x3 / stride-2 MaxPool between the Concat and this squeeze
  int64_t fire_H = 0, fire_W = 0;  //   (fire_pool_kernel / fire_pool_f16_kernel): the expands' plane and the pool window
  Window fire_pwin;
  ConvPlan plan{};        // kernel choice and weight layout for S_CONV / S_MATMUL
  float* wp = nullptr;    // packed weights (layout per plan) for S_CONV / S_MATMUL
  const int2* ktab = nullptr;  // gather table (follows wp in the packed allocation; gather kernel only)
  // f32 models (not x3, not ORE_LOAD_NO_WINOGRAD): the Winograd F(2x2, 3x3) plan of a 3x3 / stride-1 /
  // pad-1 conv (ore_conv_wino.hip), packed next to the direct one; plan() switches a conv that no
  // direct-kernel fusion takes to it
  bool has_wino = false;
  ConvPlan plan_wino{};
  float* wp_wino = nullptr;
  const float* wc1 = nullptr;  // f32 pooled first conv: weights for pooled-conv variant 7 (launch_pack_c1_f32)
  // f16 pooled first conv with the next 1x1 conv (+ Relu) fused in (conv_pair_pool_f16_kernel SQ):
  // out is that conv's output; the squeeze weights in launch_fire_pack_f16 layout
  bool c1sq = false;
  // f16 1x1 conv (+ Relu) whose only reader was GlobalAveragePool (ORE_FUSE_CONV_GAP,
  // conv1x1_gap_f16_kernel): out is the GAP's f32 [N][M] output
  bool gap = false;
  const void* sq_w = nullptr;
  const float* sq_b = nullptr;
  int64_t sq_M = 0;
  int64_t axis = 1;
  double flops_per_img = 0, bytes_per_img = 0, bytes_fixed = 0;
  double mfma_flops_per_img = -1;  // MFMA FLOPs the kernel issues when they differ from flops (Winograd)
};

}  // namespace

struct ore_model {
  ore_ctx* ctx = nullptr;
  int64_t max_batch = 0;
  int64_t run_batch = 0;         // images per pass of the graph (the arena's size; ore_model_run chunks above it)
  void* xcvt = nullptr;          // f16 F16_X_NHWC_PAIR: the f32 NCHW input converted to NHWC4 f16 (run_batch)
  size_t xcvt_bytes = 0;
  int32_t fusion = ORE_FUSE_ALL;
  bool f16 = false;              // ORE_LOAD_F16: f16 conv/pool activations, f32 accumulation
  bool wino = false;             // f32 model without ORE_LOAD_NO_WINOGRAD: Winograd plans for 3x3 s1 p1 convs
  int conv_tile = -1;            // the context's forced conv tile at load (ore_ctx_set_conv_tile)
  std::vector<Value> values;
  size_t n_base_values = 0;      // values of the graph; plan() appends views after them (pooled slices)
  std::map<std::string, int> by_name;
  std::vector<Step> base_steps;  // unfused, one per node
  std::vector<Step> steps;       // after fusion
  int input_value = -1;
  int output_value = -1;
  float* consts = nullptr;       // one device allocation for all f32 initializers
  float* packed = nullptr;       // packed conv / matmul weights (one allocation)
  std::map<int, float*> fire_packs;  // base step index -> its weights in launch_fire_pack layout
  char* arena = nullptr;        // arena_alloc + ARENA_LEAD
  char* arena_alloc = nullptr;  // the hipMalloc'd block (a 4 KiB lead before the arena proper)
  size_t arena_bytes = 0;
  // timing
  bool timing = false;
  std::vector<hipEvent_t> events;
  // branch concurrency (ore_model_set_streams): exec_steps[k] with pair_next[k] runs on the side
  // stream beside exec_steps[k + 1] (the two expand convs of a fire module: the reference's
  // branch threads, multithreading.rs:20-62)
  int streams = 1;
  std::vector<char> pair_next;
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // captured run (ore_model_graph_capture)
  hipGraph_t graph = nullptr;
  hipGraphExec_t graph_exec = nullptr;
  int timed_chunks = 0;          // image chunks of the last timed run (events: chunk x (exec_steps + 1))
  std::vector<int> exec_steps;   // indices into steps of launched (non-NOP) steps
  // run-time binding
  const float* cur_in = nullptr;
  float* cur_out = nullptr;
  bool out_bound = false;
  int64_t last_n = 0;
  bool last_chunked = false;     // the last run went in image chunks (arena values hold only the last one)
};

namespace {

bool band_step(const Step& s);      // the band walkers' geometry (below, beside step_tile_family)
bool band_f16_step(const Step& s);

// IEEE binary16 -> binary32 (exact)
float half_bits_to_float(uint16_t h) {
  const uint32_t sign = uint32_t(h & 0x8000) << 16;
  uint32_t exp = (h >> 10) & 0x1f, man = h & 0x3ff, bits;
  if (exp == 0x1f) {
    bits = sign | 0x7f800000u | (man << 13);
  } else if (exp != 0) {
    bits = sign | ((exp + 112) << 23) | (man << 13);
  } else if (man == 0) {
    bits = sign;
  } else {  // subnormal: renormalise
    int e = -1;
    do { man <<= 1; ++e; } while (!(man & 0x400));
    bits = sign | (uint32_t(112 - e) << 23) | ((man & 0x3ff) << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

ore_status err(ore_model* m, ore_status st, const std::string& msg) {
  return set_error(m->ctx, st, "%s", msg.c_str());
}

int value_id(ore_model* m, const std::string& name) {
  auto it = m->by_name.find(name);
  return it == m->by_name.end() ? -1 : it->second;
}

int new_value(ore_model* m, const std::string& name) {
  Value v;
  v.name = name;
  m->values.push_back(v);
  int id = int(m->values.size()) - 1;
  m->by_name[name] = id;  // re-definition shadows, as HashMap::insert does
  return id;
}

bool is_act(const Value& v, int rank) { return !v.is_const && v.ndim == rank; }

// ------------------------------------------------------------------ per-node shape/attr rules
ore_status build_conv(ore_model* m, const Node& n, Step* s) {
  if (n.inputs.size() < 2) return err(m, ORE_ERR_INVALID, "Conv '" + n.name + "' needs 2 inputs");
  int x = value_id(m, n.inputs[0]), w = value_id(m, n.inputs[1]);
  if (x < 0 || w < 0) return err(m, ORE_ERR_INVALID, "Conv '" + n.name + "': input not available");
  const Value &X = m->values[x], &Wt = m->values[w];
  if (!is_act(X, 4)) return err(m, ORE_ERR_UNSUPPORTED, "Conv '" + n.name + "': input must be a 4-D activation");
  if (!Wt.is_const || Wt.ndim != 4 || !Wt.cptr)
    return err(m, ORE_ERR_UNSUPPORTED, "Conv '" + n.name + "': weights must be a 4-D f32 initializer");
  int b = -1;
  if (n.inputs.size() > 2) {  // get_stored_tensor(2) (:124-130)
    b = value_id(m, n.inputs[2]);
    if (b < 0 || !m->values[b].is_const || m->values[b].ndim != 1 || !m->values[b].cptr)
      return err(m, ORE_ERR_UNSUPPORTED, "Conv '" + n.name + "': bias must be a 1-D f32 initializer");
    if (m->values[b].dims[0] != Wt.dims[0]) return err(m, ORE_ERR_INVALID, "Bias array has the wrong shape");
  }
  ore_conv_attrs a{};
  a.auto_pad = ORE_PAD_VALID;  // default (:134)
  a.group = 1;
  a.dilations[0] = a.dilations[1] = 1;
  bool have_strides = false;
  for (auto& at : n.attrs) {  // :137-163
    if (at.name == "auto_pad") {
      if (at.s == "SAME_UPPER") a.auto_pad = ORE_PAD_SAME_UPPER;
      else if (at.s == "SAME_LOWER") a.auto_pad = ORE_PAD_SAME_LOWER;
      else if (at.s == "VALID") a.auto_pad = ORE_PAD_VALID;
      else if (at.s == "NOT_SET") a.auto_pad = ORE_PAD_NOTSET;
      else return err(m, ORE_ERR_UNSUPPORTED, "Convolution Auto Pad specified not found: " + at.s);
    } else if (at.name == "dilations") {
      if (at.ints.size() < 2) return err(m, ORE_ERR_INVALID, "Conv dilations need 2 values");
      a.dilations[0] = at.ints[0]; a.dilations[1] = at.ints[1];
    } else if (at.name == "group") {
      a.group = at.i;
    } else if (at.name == "kernel_shape") {
    } else if (at.name == "pads") {
      a.n_pads = int32_t(std::min<size_t>(at.ints.size(), 4));
      for (int i = 0; i < a.n_pads; ++i) a.pads[i] = at.ints[i];
    } else if (at.name == "strides") {
      if (at.ints.size() < 2) return err(m, ORE_ERR_INVALID, "Conv strides need 2 values");
      a.strides[0] = at.ints[0]; a.strides[1] = at.ints[1];
      have_strides = true;
    } else {
      return err(m, ORE_ERR_UNSUPPORTED, "ATTRIBUTE NAME FOR CONVOLUTION NOT FOUND, " + at.name);
    }
  }
  if (!have_strides) return err(m, ORE_ERR_UNSUPPORTED, "Conv '" + n.name + "': strides attribute required");
  int64_t yd[4], p[4];
  if (ore_status st = ore_conv_out_shape(X.dims, Wt.dims, &a, yd, p)) {
    return err(m, st, "Conv '" + n.name + "': " + ore_last_error(nullptr));
  }
  s->kind = S_CONV;
  s->in0 = x; s->in1 = w; s->in2 = b;
  s->C = X.dims[1]; s->H = X.dims[2]; s->W = X.dims[3];
  s->M = Wt.dims[0]; s->kh = Wt.dims[2]; s->kw = Wt.dims[3];
  s->sh = a.strides[0]; s->sw = a.strides[1];
  s->win.pt = p[0]; s->win.pl = p[1]; s->win.pb = p[2]; s->win.pr = p[3];
  s->win.Ho = yd[2]; s->win.Wo = yd[3];
  const double P = double(yd[2] * yd[3]);
  s->flops_per_img = 2.0 * double(s->M) * P * double(s->C * s->kh * s->kw);
  const int yes = m->f16 ? 2 : 4;
  s->bytes_per_img = double(X.es) * double(s->C * s->H * s->W) + double(yes) * double(s->M) * P;
  s->bytes_fixed = double(yes) * double(Wt.numel_const()) + 4.0 * double(b >= 0 ? s->M : 0);
  int y = new_value(m, n.outputs[0]);
  Value& Y = m->values[y];
  Y.ndim = 4; Y.dims[0] = 1; Y.dims[1] = yd[1]; Y.dims[2] = yd[2]; Y.dims[3] = yd[3];
  Y.es = yes;
  s->out = y;
  return ORE_OK;
}

ore_status build_maxpool(ore_model* m, const Node& n, Step* s) {
  int x = value_id(m, n.inputs.empty() ? "" : n.inputs[0]);
  if (x < 0) return err(m, ORE_ERR_INVALID, "MaxPool '" + n.name + "': input not available");
  const Value& X = m->values[x];
  if (!is_act(X, 4)) return err(m, ORE_ERR_UNSUPPORTED, "MaxPool '" + n.name + "': input must be a 4-D activation");
  ore_pool_attrs a{};
  a.auto_pad = ORE_PAD_VALID;  // default (max_pool_op.rs:88); pads do NOT force NOTSET here
  bool have_k = false, have_s = false;
  for (auto& at : n.attrs) {  // :90-114
    if (at.name == "auto_pad") {
      if (at.s == "SAME_UPPER") a.auto_pad = ORE_PAD_SAME_UPPER;
      else if (at.s == "SAME_LOWER") a.auto_pad = ORE_PAD_SAME_LOWER;
      else if (at.s == "VALID") a.auto_pad = ORE_PAD_VALID;
      else if (at.s == "NOTSET") a.auto_pad = ORE_PAD_NOTSET;
      else return err(m, ORE_ERR_UNSUPPORTED, "MaxPool Auto Pad specified not found: " + at.s);
    } else if (at.name == "kernel_shape") {
      if (at.ints.size() < 2) return err(m, ORE_ERR_INVALID, "MaxPool kernel_shape needs 2 values");
      a.kernel[0] = at.ints[0]; a.kernel[1] = at.ints[1]; have_k = true;
    } else if (at.name == "pads") {
      a.n_pads = int32_t(std::min<size_t>(at.ints.size(), 4));
      for (int i = 0; i < a.n_pads; ++i) a.pads[i] = at.ints[i];
    } else if (at.name == "storage_order") {
    } else if (at.name == "strides") {
      if (at.ints.size() < 2) return err(m, ORE_ERR_INVALID, "MaxPool strides need 2 values");
      a.strides[0] = at.ints[0]; a.strides[1] = at.ints[1]; have_s = true;
    } else {
      return err(m, ORE_ERR_UNSUPPORTED, "ATTRIBUTE NAME FOR MAX POOL NOT FOUND, " + at.name);
    }
  }
  if (!have_k || !have_s) return err(m, ORE_ERR_UNSUPPORTED, "MaxPool '" + n.name + "': kernel_shape and strides required");
  int64_t yd[4], p[4];
  if (ore_status st = ore_pool_out_shape(X.dims, &a, yd, p))
    return err(m, st, "MaxPool '" + n.name + "': " + ore_last_error(nullptr));
  s->kind = S_MAXPOOL;
  s->in0 = x;
  s->C = X.dims[1]; s->H = X.dims[2]; s->W = X.dims[3];
  s->kh = a.kernel[0]; s->kw = a.kernel[1]; s->sh = a.strides[0]; s->sw = a.strides[1];
  s->win.pt = p[0]; s->win.pl = p[1]; s->win.pb = p[2]; s->win.pr = p[3];
  s->win.Ho = yd[2]; s->win.Wo = yd[3];
  s->bytes_per_img = double(X.es) * double(X.per_image() + s->C * yd[2] * yd[3]);
  const int xes = X.es;
  int y = new_value(m, n.outputs[0]);
  Value& Y = m->values[y];
  Y.ndim = 4; Y.dims[0] = 1; Y.dims[1] = yd[1]; Y.dims[2] = yd[2]; Y.dims[3] = yd[3];
  Y.es = xes;
  s->out = y;
  return ORE_OK;
}

ore_status build_unary4(ore_model* m, const Node& n, Step* s, StepKind kind) {
  int x = value_id(m, n.inputs.empty() ? "" : n.inputs[0]);
  if (x < 0 || !is_act(m->values[x], 4))  // `.1.clone().unwrap()` on a map entry
    return err(m, ORE_ERR_UNSUPPORTED, n.op_type + " '" + n.name + "': input must be a 4-D activation");
  s->kind = kind;
  s->in0 = x;
  const Value X = m->values[x];
  int y = new_value(m, n.outputs[0]);
  Value& Y = m->values[y];
  Y.ndim = X.ndim;
  for (int i = 0; i < 4; ++i) Y.dims[i] = X.dims[i];
  Y.es = X.es;
  s->out = y;
  s->bytes_per_img = 2.0 * X.es * double(X.per_image());
  return ORE_OK;
}

ore_status build_node(ore_model* m, const Node& n, Step* s) {
  s->op = n.op_type;
  s->name = n.name.empty() ? (n.outputs.empty() ? n.op_type : n.outputs[0]) : n.name;
  if (n.outputs.empty()) return err(m, ORE_ERR_INVALID, "node '" + n.name + "' has no outputs");
  const std::string& op = n.op_type;
  if (op == "Conv") return build_conv(m, n, s);
  if (op == "MaxPool") return build_maxpool(m, n, s);
  if (op == "Relu") return build_unary4(m, n, s, S_RELU);
  if (op == "Dropout") {  // dropout_op.rs:22-28: only `ratio`
    for (auto& at : n.attrs)
      if (at.name != "ratio") return err(m, ORE_ERR_UNSUPPORTED, "ATTRIBUTE NAME FOR DROP OUT NOT FOUND, " + at.name);
    return build_unary4(m, n, s, S_COPY);
  }
  if (op == "GlobalAveragePool") {
    ore_status st = build_unary4(m, n, s, S_GAP);
    if (st) return st;
    Value& Y = m->values[s->out];
    const Value& X = m->values[s->in0];
    Y.dims[2] = 1; Y.dims[3] = 1;
    Y.es = 4;  // f32 sums and output either way
    s->bytes_per_img = double(X.es) * double(X.per_image()) + 4.0 * double(X.dims[1]);
    return ORE_OK;
  }
  if (op == "Softmax") {  // softmax_wrapper flattens to (N, C*H*W), axis 1 (:46-51)
    ore_status st = build_unary4(m, n, s, S_SOFTMAX);
    if (st) return st;
    Value& Y = m->values[s->out];
    const Value& X = m->values[s->in0];
    Y.ndim = 2; Y.dims[0] = 1; Y.dims[1] = X.per_image(); Y.dims[2] = Y.dims[3] = 0;
    if (X.es != 4) return err(m, ORE_ERR_UNSUPPORTED, "Softmax '" + n.name + "': f16 input (f16 models end in f32 after GlobalAveragePool)");
    return ORE_OK;
  }
  if (op == "Concat") {  // concatenate_op.rs:22-32
    int64_t axis = 1;
    for (auto& at : n.attrs) {
      if (at.name != "axis") return err(m, ORE_ERR_UNSUPPORTED, "ATTRIBUTE NAME FOR CONCATENATE NOT FOUND, " + at.name);
      axis = at.i;
    }
    if (n.inputs.size() != 2) return err(m, ORE_ERR_UNSUPPORTED, "Concat '" + n.name + "': exactly 2 inputs supported");
    int a = value_id(m, n.inputs[0]), b = value_id(m, n.inputs[1]);
    if (a < 0 || b < 0 || !is_act(m->values[a], 4) || !is_act(m->values[b], 4))
      return err(m, ORE_ERR_UNSUPPORTED, "Concat '" + n.name + "': inputs must be 4-D activations");
    if (axis < 1 || axis > 3)
      return err(m, ORE_ERR_UNSUPPORTED, "Concat '" + n.name + "': axis must be 1..3 (axis 0 is the batch)");
    const Value A = m->values[a], B = m->values[b];
    for (int i = 1; i < 4; ++i)
      if (i != axis && A.dims[i] != B.dims[i]) return err(m, ORE_ERR_INVALID, "Concat '" + n.name + "': shape mismatch");
    if (A.es != B.es) return err(m, ORE_ERR_UNSUPPORTED, "Concat '" + n.name + "': inputs of different precision");
    if (A.es == 2 && axis != 1)
      return err(m, ORE_ERR_UNSUPPORTED, "Concat '" + n.name + "': f16 (channels-last) activations concatenate along axis 1 only");
    s->kind = S_CONCAT; s->in0 = a; s->in1 = b; s->axis = axis;
    int y = new_value(m, n.outputs[0]);
    Value& Y = m->values[y];
    Y.ndim = 4;
    for (int i = 0; i < 4; ++i) Y.dims[i] = A.dims[i];
    Y.dims[axis] = A.dims[axis] + B.dims[axis];
    Y.es = A.es;
    s->out = y;
    s->bytes_per_img = 2.0 * A.es * double(Y.per_image());
    return ORE_OK;
  }
  if (op == "Add") {  // add_op.rs:16-107
    if (n.inputs.size() < 2) return err(m, ORE_ERR_INVALID, "Add '" + n.name + "' needs 2 inputs");
    int a = value_id(m, n.inputs[0]), b = value_id(m, n.inputs[1]);
    if (a < 0) return err(m, ORE_ERR_INVALID, "Cannot retrieve input 1 for Add operation from hashmap input/output");
    if (b < 0 || !m->values[b].is_const || !m->values[b].cptr)
      return err(m, ORE_ERR_UNSUPPORTED, "Cannot retrieve input 2 for Add operation");
    const Value A = m->values[a], B = m->values[b];
    if (A.is_const) return err(m, ORE_ERR_UNSUPPORTED, "Add '" + n.name + "': constant first input not supported");
    if (A.es != 4) return err(m, ORE_ERR_UNSUPPORTED, "Add '" + n.name + "': f16 input is not supported (f32 op)");
    if (!((A.ndim == 4 && B.ndim == 3) || (A.ndim == 2 && B.ndim == 2)))
      return err(m, ORE_ERR_UNSUPPORTED, "Add '" + n.name + "': supports 4-D + 3-D or 2-D + 2-D");
    for (int i = 0; i < B.ndim; ++i) {  // right-aligned broadcast; the batch axis of A is 1 here
      const int ai = A.ndim - B.ndim + i;
      const int64_t ad = A.dims[ai];
      if (B.dims[i] != 1 && B.dims[i] != ad && !(ai == 0 && B.dims[i] == 1))
        return err(m, ORE_ERR_INVALID, "Add '" + n.name + "': shapes not broadcastable");
      if (ai == 0 && B.dims[i] != 1)
        return err(m, ORE_ERR_UNSUPPORTED, "Add '" + n.name + "': constant may not span the batch axis");
    }
    s->kind = S_ADD; s->in0 = a; s->in1 = b;
    int y = new_value(m, n.outputs[0]);
    Value& Y = m->values[y];
    Y.ndim = A.ndim;
    for (int i = 0; i < 4; ++i) Y.dims[i] = A.dims[i];
    s->out = y;
    s->bytes_per_img = 8.0 * double(A.per_image());
    return ORE_OK;
  }
  if (op == "Reshape") {  // reshape_op.rs:16-92
    if (n.inputs.size() < 2) return err(m, ORE_ERR_INVALID, "Reshape '" + n.name + "' needs 2 inputs");
    int x = value_id(m, n.inputs[0]), sh = value_id(m, n.inputs[1]);
    if (x < 0) return err(m, ORE_ERR_INVALID, "Reshape '" + n.name + "': input not available");
    if (sh < 0 || !m->values[sh].is_const || !m->values[sh].has_i64)
      return err(m, ORE_ERR_UNSUPPORTED, "Unable to retrieve Shape for Reshape operation");
    const Value X = m->values[x];
    const std::vector<int64_t> shape = m->values[sh].i64;
    if (X.ndim != 4) return err(m, ORE_ERR_UNSUPPORTED, "Reshape '" + n.name + "': data must be 4-D");
    if (shape.size() < 2) return err(m, ORE_ERR_UNSUPPORTED, "Reshape '" + n.name + "': shape must have 2 values");
    int64_t ns[2] = {shape[0], shape[1]};
    for (int i = 0; i < 2; ++i)
      if (ns[i] == 0) ns[i] = X.dims[i];
    if (ns[0] < 0 || ns[1] < 0) return err(m, ORE_ERR_UNSUPPORTED, "Reshape '" + n.name + "': negative dims");
    if (X.is_const) {  // fold: a reinterpretation of the uploaded initializer
      if (ns[0] * ns[1] != X.numel_const()) return err(m, ORE_ERR_INVALID, "Reshape: element count mismatch");
      int y = new_value(m, n.outputs[0]);
      Value& Y = m->values[y];
      Y.is_const = true; Y.ndim = 2; Y.dims[0] = ns[0]; Y.dims[1] = ns[1]; Y.cptr = m->values[x].cptr;
      s->kind = S_NOP;
      s->out = y;
      return ORE_OK;
    }
    if (ns[0] != 1 || ns[1] != X.per_image())
      return err(m, ORE_ERR_UNSUPPORTED, "Reshape '" + n.name + "': activation reshape must be [1 or 0, C*H*W] per image");
    if (X.es == 2 && X.dims[2] * X.dims[3] != 1)
      return err(m, ORE_ERR_UNSUPPORTED, "Reshape '" + n.name + "': f16 activations are channels-last; flattening one is not supported");
    s->kind = S_COPY; s->in0 = x;
    int y = new_value(m, n.outputs[0]);
    Value& Y = m->values[y];
    Y.ndim = 2; Y.dims[0] = 1; Y.dims[1] = ns[1];
    Y.es = X.es;
    s->out = y;
    s->bytes_per_img = 8.0 * double(X.per_image());
    return ORE_OK;
  }
  if (op == "MatMul") {  // mul_op.rs:11-32: both operands Array2 from the map
    if (n.inputs.size() < 2) return err(m, ORE_ERR_INVALID, "MatMul '" + n.name + "' needs 2 inputs");
    int a = value_id(m, n.inputs[0]), b = value_id(m, n.inputs[1]);
    if (a < 0 || b < 0) return err(m, ORE_ERR_INVALID, "MatMul '" + n.name + "': input not available");
    const Value A = m->values[a], B = m->values[b];
    if (A.ndim != 2 || B.ndim != 2) return err(m, ORE_ERR_UNSUPPORTED, "MatMul '" + n.name + "': operands must be 2-D");
    if (A.is_const || !B.is_const || !B.cptr)
      return err(m, ORE_ERR_UNSUPPORTED, "MatMul '" + n.name + "': expects activation . constant");
    if (A.dims[1] != B.dims[0]) return err(m, ORE_ERR_INVALID, "MatMul '" + n.name + "': inner dims differ");
    if (A.es != 4) return err(m, ORE_ERR_UNSUPPORTED, "MatMul '" + n.name + "': f16 input is not supported (f32 op)");
    s->kind = S_MATMUL; s->in0 = a; s->in1 = b;
    s->C = A.dims[1]; s->M = B.dims[1]; s->w_kmajor = true;
    s->win.Ho = 1; s->win.Wo = 1; s->H = 1; s->W = 1; s->kh = 1; s->kw = 1;
    s->flops_per_img = 2.0 * double(A.dims[1] * B.dims[1]);
    s->bytes_per_img = 4.0 * double(A.dims[1] + B.dims[1]);
    s->bytes_fixed = 4.0 * double(B.numel_const());
    int y = new_value(m, n.outputs[0]);
    Value& Y = m->values[y];
    Y.ndim = 2; Y.dims[0] = 1; Y.dims[1] = B.dims[1];
    s->out = y;
    return ORE_OK;
  }
  return err(m, ORE_ERR_UNSUPPORTED, "INFERENCE OPERATION '" + op + "' NOT FOUND FOR NODE " + n.name);
}

// ------------------------------------------------------------------ fusion + planning
// plan() rewrites the unfused node steps (base_steps) into the launched plan in passes, each a
// pattern over the step list that turns a producer -> consumer chain into one kernel step (the
// consumer steps become S_NOP, the values between them `elided`).  Every fusion is exact: the fused
// kernels keep each output's arithmetic (same operands, same k order, the max of the same values),
// so the result of the graph does not depend on which passes ran (tests/test_model_gpu.py checks each
// against the unfused graph bit for bit).  Pass order matters only where two patterns overlap
// (fire + pool + squeeze before concat + pool).  Then: algorithm selection (Winograd), aliases,
// Concat in place, the plane layout, the arena, branch pairs and the gather tables.
void count_uses(ore_model* m, const std::vector<Step>& steps) {
  for (auto& v : m->values) v.uses = 0;
  for (auto& s : steps)
    for (int id : {s.in0, s.in1, s.in2, s.in3})
      if (id >= 0) m->values[id].uses++;
}

// plane stride of a padded activation: 128-B aligned planes when that costs <= 5 %, else 16-B
// aligned ones when that does (13 x 13 -> 172: the streaming conv's 16-B operand loads and stores
// need 4-float planes), else dense
int64_t padded_plane(int64_t P) {
  int64_t Pp = (P + 31) / 32 * 32;
  if (Pp - P > P / 20) Pp = (P + 3) / 4 * 4;
  return Pp - P <= P / 20 ? Pp : P;
}

bool strided_writer(const Step& s) { return s.kind == S_CONV || s.kind == S_FIRE || s.kind == S_MAXPOOL; }

// size heuristics of the fusion passes (measured at batch 256, DESIGN.md sections 3 and 7); ORE_FUSE_EAGER
// (tests) applies every eligible fusion regardless
constexpr int64_t FIRE_MIN_COLS = 65536;      // fire fusions: max_batch x H x W >= one 64-pixel wave per SIMD
constexpr int64_t FIRE_POOL_MIN_HW = 1024;    // fire + pool + squeeze on 54 x 54 planes (at 27 x 27 Winograd wins)
constexpr int64_t CONCAT_POOL_MIN_HW = 1024;  // concat + pool in the producers: fire4 -40 us, fire8 +21 us
constexpr double EPOOL_MAX_WORK = 1.25;       // conv + pool patch kernel: recomputed columns <= 1.25 x the conv's
constexpr int64_t WINO_SPLIT_MIN_C = 48;      // fire + squeeze on planes < FIRE_POOL_MIN_HW with >= 48 squeeze
                                              // channels: expand1x1 + Winograd expand3x3 + squeeze as three launches
                                              // (fire6 / fire7: 328 / 323 us vs 345 / 362 fused; fire5 at C = 32: 192 vs 173)

struct Planner {
  ore_model* m;
  std::vector<int> producer;  // value -> the step that writes it (-1: input / constant)
  bool eager() const { return (m->fusion & ORE_FUSE_EAGER) != 0; }
  bool has(int32_t flags) const { return (m->fusion & flags) == flags; }
  Step& st(int i) { return m->steps[i]; }
  Value& val(int i) { return m->values[i]; }
  // the first launched step at or after `from` that reads v (in0 or in1)
  int reader(int v, size_t from) const {
    for (size_t j = from; j < m->steps.size(); ++j)
      if (m->steps[j].kind != S_NOP && (m->steps[j].in0 == v || m->steps[j].in1 == v || m->steps[j].in3 == v))
        return int(j);
    return -1;
  }
  // a value read once, not the graph output: free to elide
  bool private_value(int v) const { return m->values[v].uses == 1 && !m->values[v].is_output; }
  void nop(Step& s) {
    s.kind = S_NOP;
    s.in0 = s.in1 = s.in3 = -1;
  }
  void recount() { count_uses(m, m->steps); }
  // a plain f32 1x1 conv (+ Relu) on the direct kernels, output the size of its input
  static bool plain_1x1(const Step& s) {
    return s.kind == S_CONV && s.relu && !s.pool && !s.epool && !s.plan.f16 && s.kh == 1 && s.kw == 1 && s.sh == 1 &&
           s.sw == 1 && s.win.pt == 0 && s.win.pl == 0 && s.win.Ho == s.H && s.win.Wo == s.W;
  }
  // an f32 3x3 / stride-1 'same' conv (+ Relu) on the direct kernels
  static bool same_3x3(const Step& s) {
    return s.kind == S_CONV && s.relu && !s.pool && !s.epool && !s.plan.f16 && s.kh == 3 && s.kw == 3 && s.sh == 1 &&
           s.sw == 1 && s.win.pt == 1 && s.win.pl == 1 && s.win.Ho == s.H && s.win.Wo == s.W;
  }
  // a weight packing made once per model (fire_packs[key]); false on an allocation failure
  template <class F>
  bool pack_once(int key, size_t bytes, F launch) {
    if (m->fire_packs.count(key)) return true;
    float* buf = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&buf), bytes) != hipSuccess) return false;
    launch(buf);
    m->fire_packs[key] = buf;
    return hipGetLastError() == hipSuccess && hipStreamSynchronize(m->ctx->stream) == hipSuccess;
  }
  // the fire modules: Concat step i of two producers (e1 a 1x1, e3 a 3x3 'same' conv of one value S)
  bool fire_concat(int i, int* pa, int* pb) {
    const Step& cc = st(i);
    if (cc.kind != S_CONCAT || cc.axis != 1 || cc.in0 < 0 || cc.in1 < 0 || cc.in0 == cc.in1) return false;
    *pa = producer[cc.in0];
    *pb = producer[cc.in1];
    return *pa >= 0 && *pb >= 0 && *pa != *pb;
  }

  // MaxPool step pl (3x3 / stride 2, f32 NCHW input) feeding 1x1 conv cv fits pool_conv1x1_f32_kernel
  bool pool_squeeze_fits(const Step& pl, const Step& cv) const {
    if (pl.kind != S_MAXPOOL || pl.kh != 3 || pl.kw != 3 || pl.sh != 2 || pl.sw != 2) return false;
    if (m->values[pl.in0].es != 4 || m->values[pl.in0].nhwc) return false;
    if (cv.kind != S_CONV || cv.pool || cv.epool || cv.kh != 1 || cv.kw != 1 || cv.sh != 1 || cv.sw != 1 ||
        cv.win.pt || cv.win.pl || cv.plan.f16 || cv.plan.wino || cv.M > 64 || cv.C % 32 ||
        pl.win.pt > 2 || pl.win.pl > 2)
      return false;
    PoolConvParams q{};  // pool_conv1x1_f32_kernel's own limits (run_conv_pool has no other kernel)
    q.C = int(cv.C); q.H = int(pl.H); q.W = int(pl.W); q.Hp = int(pl.win.Ho); q.Wp = int(pl.win.Wo);
    q.pt = int(pl.win.pt); q.pl = int(pl.win.pl); q.M = int(cv.M); q.Mp = cv.plan.Mp; q.Kp = cv.plan.krows;
    q.N = 1; q.x_ps = int(pl.H * pl.W); q.y_ps = int(pl.win.Ho * pl.win.Wo);
    q.x_nstride = int64_t(q.C) * q.x_ps; q.y_nstride = int64_t(q.M) * q.y_ps;
    return pool_conv1x1_f32_eligible(q);
  }
  // Winograd models: a fire module -> MaxPool -> squeeze runs cheaper as expand1x1 + Winograd
  // expand3x3 + the pooled squeeze (pool_squeeze) than in the direct-kernel fusions (fire4 -> pool3
  // -> fire5: 105 + 344 + pool and squeeze vs 713 us fused, profiles/r03_fusion_split.txt)
  bool wino_pool_split(const Step& e3, const Step& pl, int qi) const {
    return !eager() && m->wino && e3.has_wino && has(ORE_FUSE_POOL_SQUEEZE) && qi >= 0 &&
           private_value(pl.out) && m->steps[qi].in0 == pl.out && pool_squeeze_fits(pl, m->steps[qi]);
  }

  // (1) Conv -> Relu: the Relu in the conv epilogue
  void conv_relu() {
    if (!has(ORE_FUSE_CONV_RELU)) return;
    for (size_t i = 0; i < m->steps.size(); ++i) {
      Step& r = st(int(i));
      if (r.kind != S_RELU) continue;
      const int v = r.in0, p = producer[v];
      if (p < 0 || st(p).kind != S_CONV || st(p).relu || !private_value(v)) continue;
      st(p).out = r.out;
      st(p).relu = true;
      val(v).elided = true;
      producer[r.out] = p;
      nop(r);
    }
    recount();
  }

  // (2) Conv (-> Relu) -> MaxPool, the conv output read by the pool only: one launch when the
  // recomputed patch costs <= EPOOL_MAX_WORK x the conv's columns (f32 and f16 models)
  ore_status conv_pool() {
    if (!has(ORE_FUSE_CONV_POOL)) return ORE_OK;
    for (size_t i = 0; i < m->steps.size(); ++i) {
      Step& pl = st(int(i));
      if (pl.kind != S_MAXPOOL) continue;
      const int v = pl.in0, pc = producer[v];
      if (pc < 0 || !private_value(v)) continue;
      Step& cv = st(pc);
      if (cv.kind != S_CONV || cv.pool || cv.epool) continue;
      if (cv.plan.f16 != (val(pl.out).es == 2 ? 1 : 0)) continue;  // f16 conv -> f16 pool only
      int a = 0, b = 0;
      const double work = epool_tile(cv.win.Ho, cv.win.Wo, pl.kh, pl.kw, pl.sh, pl.sw, pl.win, &a, &b);
      if (work == 0.0 || (work > EPOOL_MAX_WORK && !eager())) continue;
      cv.epool = true;
      cv.out = pl.out;
      // f32: pack the weights for the window kernel (pooled-conv variant 7) when its geometry fits
      if (!cv.plan.f16 && cv.kh == 7 && cv.kw == 7 && cv.sh == 2 && cv.sw == 2 && cv.in1 >= 0 &&
          (cv.C == 1 || cv.C == 3 || cv.C == 4) && cv.M > 32 && cv.M <= 128) {
        const int key = 4000000 + pc, K = int(cv.C * cv.kh * cv.kw), M = int(cv.M);
        const float* w = val(cv.in1).cptr;
        if (!pack_once(key, c1_f32_pack_bytes(M, K), [&](float* buf) { launch_pack_c1_f32(w, M, K, buf, m->ctx->stream); }))
          return err(m, ORE_ERR_HIP, "conv weight packing failed");
        cv.wc1 = m->fire_packs[key];
      }
      cv.ep_kh = pl.kh; cv.ep_kw = pl.kw; cv.ep_sh = pl.sh; cv.ep_sw = pl.sw; cv.ep_win = pl.win;
      // algorithmic bytes: the conv's input + the pooled output (the pre-pool tensor never moves)
      cv.bytes_per_img = double(val(cv.in0).es) * double(cv.C * cv.H * cv.W) +
                         double(val(pl.out).es) * double(cv.M * pl.win.Ho * pl.win.Wo);
      val(v).elided = true;
      producer[pl.out] = pc;
      nop(pl);
    }
    recount();
    return ORE_OK;
  }

  // (3) f32 fire module -> 3x3 / stride-2 MaxPool -> the next squeeze in one fire_pool_kernel launch
  // (ore_fire.hip): Concat(e1 1x1, e3 3x3 'same') (+ Relu), the pool the Concat's only reader, the
  // squeeze (1x1 + Relu, <= 64 channels) the pool's only reader.  Expand planes of >= FIRE_POOL_MIN_HW
  // pixels (SqueezeNet's fire4 -> pool3 -> fire5; at 27 x 27 fire8's expand3x3 runs Winograd, cheaper
  // than the direct K loop).  Runs before concat_pool, which would otherwise take the pattern.
  ore_status fire_pool_f32() {
    if (!has(ORE_FUSE_FIRE_POOL | ORE_FUSE_CONV_RELU | ORE_FUSE_CONCAT) || m->f16) return ORE_OK;
    for (size_t i = 0; i < m->steps.size(); ++i) {
      int pa, pb;
      if (!fire_concat(int(i), &pa, &pb)) continue;
      Step& cc = st(int(i));
      const int pi = reader(cc.out, i + 1);
      if (pi < 0) continue;
      Step& pl = st(pi);
      if (pl.kind != S_MAXPOOL || pl.kh != 3 || pl.kw != 3 || pl.sh != 2 || pl.sw != 2 || pl.in0 != cc.out) continue;
      const int qi = reader(pl.out, size_t(pi) + 1);
      if (qi < 0) continue;
      Step &e1 = st(pa), &e3 = st(pb), &q = st(qi);
      if (!plain_1x1(e1) || !same_3x3(e3) || !plain_1x1(q) || q.in0 != pl.out || e1.in0 != e3.in0 || e1.H != e3.H ||
          e1.W != e3.W)
        continue;
      if (e1.M % 64 || e3.M % 64 || q.M > 64 || e1.C % 16 || q.C != e1.M + e3.M || pl.H != e1.H || pl.W != e1.W) continue;
      if (!eager() && (e1.H * e1.W < FIRE_POOL_MIN_HW || m->max_batch * e1.H * e1.W < FIRE_MIN_COLS)) continue;
      if (wino_pool_split(e3, pl, qi)) continue;
      if (q.in2 < 0 || e1.in2 < 0 || e3.in2 < 0 || padded_plane(e1.H * e1.W) % 4) continue;  // 16-B input planes
      FireParams fp{};
      fp.H = int(e1.H); fp.W = int(e1.W);
      fp.Hp = int(pl.win.Ho); fp.Wp = int(pl.win.Wo); fp.ppt = int(pl.win.pt); fp.ppl = int(pl.win.pl);
      if (!fire_pool_plan(&fp) || fp.ppt > 2 || fp.ppl > 2 || 2 * (fp.Hp - 1) - fp.ppt >= fp.H ||
          2 * (fp.Wp - 1) - fp.ppl >= fp.W)
        continue;
      if (!private_value(cc.in0) || !private_value(cc.in1) || !private_value(cc.out) || !private_value(pl.out) ||
          val(e1.in0).es != 4)
        continue;
      for (int idx : {pa, pb}) {  // the fire kernel's row-permuted expand packings (shared with fire_f32)
        const Step& e = st(idx);
        const int64_t K = e.C * e.kh * e.kw, Kp = (K + 31) / 32 * 32;
        const float* w = val(e.in1).cptr;
        if (!pack_once(idx, size_t(Kp * e.M) * 4,
                       [&](float* buf) { launch_fire_pack(w, int(e.M), int(K), buf, m->ctx->stream); }))
          return err(m, ORE_ERR_HIP, "fire weight packing failed");
      }
      q.kind = S_FIRE;
      q.fire_pool = true;
      q.fire_H = e1.H;
      q.fire_W = e1.W;
      q.fire_pwin = pl.win;
      q.in0 = e1.in0;
      q.fire_C = e1.C;
      q.fire_E1 = e1.M;
      q.fire_E3 = e3.M;
      q.fire_w1 = m->fire_packs[pa];
      q.fire_w3 = m->fire_packs[pb];
      q.fire_b1 = val(e1.in2).cptr;
      q.fire_b3 = val(e3.in2).cptr;
      q.flops_per_img += e1.flops_per_img + e3.flops_per_img;
      q.bytes_per_img = 4.0 * double(e1.C * e1.H * e1.W) + 4.0 * double(q.M * q.H * q.W);
      q.name = e1.name.substr(0, e1.name.find('/')) + "+pool+" + q.name;
      val(cc.in0).elided = val(cc.in1).elided = val(cc.out).elided = val(pl.out).elided = true;
      nop(e1); nop(e3); nop(cc); nop(pl);
    }
    recount();
    return ORE_OK;
  }

  // (4) Concat(e1, e3) -> 3x3 / stride-2 MaxPool, e1 / e3 Convs (+ Relu) read only by the Concat (f32):
  // each conv's pooled epilogue writes its channel slice of the pool output (a view appended to the
  // values), so neither the two conv outputs nor the concat reach HBM.  The MaxPool of a Concat is the
  // Concat of the per-slice MaxPools (the pool is per channel).  Conv planes of >= CONCAT_POOL_MIN_HW.
  void concat_pool() {
    if (!has(ORE_FUSE_CONCAT_POOL | ORE_FUSE_CONV_POOL | ORE_FUSE_CONCAT) || m->f16) return;
    for (size_t i = 0; i < m->steps.size(); ++i) {
      Step& pl = st(int(i));
      if (pl.kind != S_MAXPOOL || pl.kh != 3 || pl.kw != 3 || pl.sh != 2 || pl.sw != 2) continue;
      const int cv = pl.in0, ci = producer[cv];
      if (ci < 0 || !private_value(cv) || val(pl.out).is_output) continue;
      int pa, pb;
      if (!fire_concat(ci, &pa, &pb)) continue;
      Step& cc = st(ci);
      auto ok = [&](const Step& s, int v) {
        return s.kind == S_CONV && s.relu && !s.pool && !s.epool && !s.plan.f16 && private_value(v) && val(v).ndim == 4;
      };
      if (!ok(st(pa), cc.in0) || !ok(st(pb), cc.in1)) continue;
      int t1 = 0, t2 = 0;
      const Step& sa = st(pa);
      if (epool_tile(sa.win.Ho, sa.win.Wo, pl.kh, pl.kw, pl.sh, pl.sw, pl.win, &t1, &t2) == 0.0) continue;
      if (sa.win.Ho * sa.win.Wo < CONCAT_POOL_MIN_HW && !eager()) continue;
      if (wino_pool_split(st(pb), pl, reader(pl.out, i + 1))) continue;
      const int pout = pl.out;
      const int64_t Hp = val(pout).dims[2], Wp = val(pout).dims[3];
      const int pes = val(pout).es;
      const std::string pname = val(pout).name;
      int64_t ch0 = 0;
      for (int half = 0; half < 2; ++half) {
        const int si = half ? pb : pa, src = half ? cc.in1 : cc.in0;
        Value v;
        v.name = pname + (half ? "#slice1" : "#slice0");
        v.ndim = 4;
        v.dims[0] = 1; v.dims[1] = val(src).dims[1]; v.dims[2] = Hp; v.dims[3] = Wp;
        v.es = pes;
        v.alias_of = pout; v.alias_ch = ch0; v.slice = true;
        ch0 += v.dims[1];
        m->values.push_back(v);
        producer.push_back(si);
        const int vid = int(m->values.size()) - 1;
        Step& s = st(si);
        val(src).elided = true;
        s.epool = true;
        s.out = vid;
        s.ep_kh = pl.kh; s.ep_kw = pl.kw; s.ep_sh = pl.sh; s.ep_sw = pl.sw; s.ep_win = pl.win;
        s.bytes_per_img = double(val(s.in0).es) * double(s.C * s.H * s.W) + double(pes) * double(s.M * Hp * Wp);
      }
      val(cv).elided = true;
      producer[pout] = pa;
      nop(cc);
      nop(pl);
    }
    recount();
  }

  // (5) fire module + the next squeeze in one launch (f32, fire_kernel): Concat(e1, e3) whose inputs
  // are a 1x1 and a 3x3 'same' Conv (+ Relu) of one value S, read only by a 1x1 Conv (+ Relu) with at
  // most 64 output channels
  ore_status fire_f32() {
    if (!has(ORE_FUSE_FIRE | ORE_FUSE_CONV_RELU | ORE_FUSE_CONCAT) || m->f16) return ORE_OK;
    for (size_t i = 0; i < m->steps.size(); ++i) {
      int pa, pb;
      if (!fire_concat(int(i), &pa, &pb)) continue;
      Step& cc = st(int(i));
      const int qi = reader(cc.out, i + 1);
      if (qi < 0) continue;
      Step &e1 = st(pa), &e3 = st(pb), &q = st(qi);
      if (!plain_1x1(e1) || !same_3x3(e3) || !plain_1x1(q) || q.in0 != cc.out || e1.in0 != e3.in0 || e1.H != e3.H ||
          e1.W != e3.W)
        continue;
      if (e1.M % 64 || e3.M % 64 || q.M > 64 || e1.C % 16 || q.C != e1.M + e3.M) continue;
      if (!eager() && m->max_batch * e1.H * e1.W < FIRE_MIN_COLS) continue;
      // Winograd expand3x3 (f32 models with Winograd on): the split is cheaper on small planes with wide inputs
      if (!eager() && m->wino && e3.has_wino && e1.H * e1.W < FIRE_POOL_MIN_HW && e1.C >= WINO_SPLIT_MIN_C) continue;
      if (padded_plane(e1.H * e1.W) % 4) continue;  // 16-B planes (layout below)
      if (!private_value(cc.in0) || !private_value(cc.in1) || !private_value(cc.out) || val(e1.in0).es != 4) continue;
      if (e1.in2 < 0 || e3.in2 < 0 || q.in2 < 0) continue;
      for (int idx : {pa, pb}) {
        const Step& e = st(idx);
        const int64_t K = e.C * e.kh * e.kw, Kp = (K + 31) / 32 * 32;
        const float* w = val(e.in1).cptr;
        if (!pack_once(idx, size_t(Kp * e.M) * 4,
                       [&](float* buf) { launch_fire_pack(w, int(e.M), int(K), buf, m->ctx->stream); }))
          return err(m, ORE_ERR_HIP, "fire weight packing failed");
      }
      q.kind = S_FIRE;
      q.in0 = e1.in0;
      q.fire_C = e1.C;
      q.fire_E1 = e1.M;
      q.fire_E3 = e3.M;
      q.fire_w1 = m->fire_packs[pa];
      q.fire_w3 = m->fire_packs[pb];
      q.fire_b1 = val(e1.in2).cptr;
      q.fire_b3 = val(e3.in2).cptr;
      q.flops_per_img += e1.flops_per_img + e3.flops_per_img;
      q.bytes_per_img = 4.0 * double(e1.C * e1.H * e1.W) + 4.0 * double(q.M * q.H * q.W);
      q.name = e1.name.substr(0, e1.name.find('/')) + "+" + q.name;
      val(cc.in0).elided = val(cc.in1).elided = val(cc.out).elided = true;
      nop(e1); nop(e3); nop(cc);
    }
    recount();
    return ORE_OK;
  }

  // (6) f16 models: the same fire module + next squeeze pattern in one fire_f16_kernel launch
  // (ore_fire_f16.hip): expand1x1 / expand3x3 (+ Relu) on 16-B NHWC gathers, C % 16 == 0 and <= 64,
  // expands in 32-channel chunks, the squeeze <= 64 channels; bit-identical to the three
  // conv_f16_kernel launches.  With a 3x3 / stride-2 MaxPool between the Concat and the squeeze
  // (SqueezeNet fire4 -> pool3 -> fire5, fire8 -> pool5 -> fire9) the pooled kernel takes all four
  // steps (ORE_FUSE_FIRE_POOL; bit-identical to the three convs + maxpool_nhwc_kernel)
  ore_status fire_f16() {
    if (!has(ORE_FUSE_FIRE | ORE_FUSE_CONV_RELU) || !m->f16) return ORE_OK;
    const bool pooled = has(ORE_FUSE_FIRE_POOL);
    for (size_t i = 0; i < m->steps.size(); ++i) {
      int pa, pb;
      if (!fire_concat(int(i), &pa, &pb)) continue;
      Step& cc = st(int(i));
      int qi = reader(cc.out, i + 1), pi = -1;
      if (qi < 0) continue;
      if (st(qi).kind == S_MAXPOOL) {  // pooled form: Concat -> 3x3 / stride-2 MaxPool (read once) -> squeeze
        const Step& pl = st(qi);
        if (!pooled || pl.kh != 3 || pl.kw != 3 || pl.sh != 2 || pl.sw != 2 || pl.in0 != cc.out) continue;
        if (!private_value(pl.out)) continue;
        pi = qi;
        qi = reader(pl.out, size_t(pi) + 1);
        if (qi < 0) continue;
      }
      const int qin = pi >= 0 ? st(pi).out : cc.out;
      Step &e1 = st(pa), &e3 = st(pb), &q = st(qi);
      auto vec16 = [](const Step& s) {
        return s.kind == S_CONV && s.relu && !s.pool && !s.epool && s.plan.f16 && s.plan.xmode == F16_X_NHWC_VEC &&
               s.sh == 1 && s.sw == 1 && s.win.Ho == s.H && s.win.Wo == s.W;
      };
      auto is1x1 = [&](const Step& s) { return vec16(s) && s.kh == 1 && s.kw == 1 && s.win.pt == 0 && s.win.pl == 0; };
      const bool e3ok = vec16(e3) && e3.kh == 3 && e3.kw == 3 && e3.win.pt == 1 && e3.win.pl == 1;
      if (!is1x1(e1) || !e3ok || !is1x1(q) || q.in0 != qin || e1.in0 != e3.in0 || e1.H != e3.H || e1.W != e3.W) continue;
      if (e1.C % 16 || e1.C > 64 || e1.M % 32 || e3.M % 32 || q.M % 8 || q.M > 64 || q.C != e1.M + e3.M) continue;
      if (q.in2 < 0 || e1.in2 < 0 || e3.in2 < 0) continue;
      if (pi < 0 && fire_f16_lds_bytes(int(e1.C), int(e1.H), int(e1.W)) > FIRE_F16_LDS_MAX) continue;
      if (pi >= 0) {  // a band shape must fit (fire_pool_f16_plan) and every window touch the image
        const Step& pl = st(pi);
        FireF16Params fp{};
        fp.C = int(e1.C); fp.H = int(e1.H); fp.W = int(e1.W);
        fp.Hp = int(pl.win.Ho); fp.Wp = int(pl.win.Wo); fp.ppt = int(pl.win.pt); fp.ppl = int(pl.win.pl);
        if (pl.H != e1.H || pl.W != e1.W || !fire_pool_f16_plan(&fp) || pl.win.pt > 2 || pl.win.pl > 2 ||
            2 * (fp.Hp - 1) - fp.ppt >= fp.H || 2 * (fp.Wp - 1) - fp.ppl >= fp.W)
          continue;
      }
      if (!private_value(cc.in0) || !private_value(cc.in1) || !private_value(cc.out) || val(e1.in0).es != 2) continue;
      // the three weight packings (made once per model; keys 2000000 + expand index, 3000000 + squeeze index)
      for (int idx : {pa, pb, qi}) {
        const Step& e = st(idx);
        const int kk = int(e.kh * e.kw), M = int(e.M), C = int(e.C);
        const float* w = val(e.in1).cptr;
        if (!pack_once((idx == qi ? 3000000 : 2000000) + idx, fire_pack_f16_bytes(M, C, kk),
                       [&](float* buf) { launch_fire_pack_f16(w, M, C, kk, buf, m->ctx->stream); }))
          return err(m, ORE_ERR_HIP, "f16 fire weight packing failed");
      }
      q.kind = S_FIRE;
      q.fire_f16 = true;
      q.fire_pool = pi >= 0;
      q.fire_H = e1.H;
      q.fire_W = e1.W;
      if (pi >= 0) {
        Step& pl = st(pi);
        q.fire_pwin = pl.win;
        val(pl.out).elided = true;
        nop(pl);
      }
      q.in0 = e1.in0;
      q.fire_C = e1.C;
      q.fire_E1 = e1.M;
      q.fire_E3 = e3.M;
      q.fire_w1 = m->fire_packs[2000000 + pa];
      q.fire_w3 = m->fire_packs[2000000 + pb];
      q.fire_ws16 = m->fire_packs[3000000 + qi];
      q.fire_b1 = val(e1.in2).cptr;
      q.fire_b3 = val(e3.in2).cptr;
      q.flops_per_img += e1.flops_per_img + e3.flops_per_img;
      q.bytes_per_img = 2.0 * double(e1.C * e1.H * e1.W) + 2.0 * double(q.M * q.H * q.W);
      q.name = e1.name.substr(0, e1.name.find('/')) + (pi >= 0 ? "+pool+" : "+") + q.name;
      val(cc.in0).elided = val(cc.in1).elided = val(cc.out).elided = true;
      nop(e1); nop(e3); nop(cc);
    }
    recount();
    return ORE_OK;
  }

  // (6b) f16 models: a fire module whose Concat no squeeze takes (SqueezeNet fire9, read by conv10):
  // expand1x1 + expand3x3 (+ Relu) + Concat in one fire_f16_kernel<NKC, 0> launch that writes the
  // Concat (NHWC) -- the two conv_f16 launches' arithmetic, bit-identical
  ore_status fire_f16_concat() {
    if (!has(ORE_FUSE_FIRE | ORE_FUSE_CONV_RELU) || !m->f16) return ORE_OK;
    for (size_t i = 0; i < m->steps.size(); ++i) {
      int pa, pb;
      if (!fire_concat(int(i), &pa, &pb)) continue;
      Step& cc = st(int(i));
      Step &e1 = st(pa), &e3 = st(pb);
      auto vec16 = [](const Step& s) {
        return s.kind == S_CONV && s.relu && !s.pool && !s.epool && s.plan.f16 && s.plan.xmode == F16_X_NHWC_VEC &&
               s.sh == 1 && s.sw == 1 && s.win.Ho == s.H && s.win.Wo == s.W;
      };
      const bool e1ok = vec16(e1) && e1.kh == 1 && e1.kw == 1 && e1.win.pt == 0 && e1.win.pl == 0;
      const bool e3ok = vec16(e3) && e3.kh == 3 && e3.kw == 3 && e3.win.pt == 1 && e3.win.pl == 1;
      if (!e1ok || !e3ok || e1.in0 != e3.in0 || e1.H != e3.H || e1.W != e3.W || e1.C != e3.C) continue;
      if (e1.C % 16 || e1.C > 64 || e1.M % 32 || e3.M % 32 || e1.M + e3.M > 512 || e1.in2 < 0 || e3.in2 < 0) continue;
      if (fire_f16_lds_bytes(int(e1.C), int(e1.H), int(e1.W)) > FIRE_F16_LDS_MAX) continue;
      if (!private_value(cc.in0) || !private_value(cc.in1) || val(e1.in0).es != 2) continue;
      for (int idx : {pa, pb}) {
        const Step& e = st(idx);
        const int kk = int(e.kh * e.kw), M = int(e.M), C = int(e.C);
        const float* w = val(e.in1).cptr;
        if (!pack_once(2000000 + idx, fire_pack_f16_bytes(M, C, kk),
                       [&](float* buf) { launch_fire_pack_f16(w, M, C, kk, buf, m->ctx->stream); }))
          return err(m, ORE_ERR_HIP, "f16 fire weight packing failed");
      }
      cc.kind = S_FIRE;
      cc.fire_f16 = true;
      cc.fire_pool = false;
      cc.fire_H = e1.H;
      cc.fire_W = e1.W;
      cc.H = e1.H;
      cc.W = e1.W;
      cc.M = 0;  // no squeeze: the Concat is the output
      cc.in0 = e1.in0;
      cc.in1 = cc.in2 = -1;
      cc.fire_C = e1.C;
      cc.fire_E1 = e1.M;
      cc.fire_E3 = e3.M;
      cc.fire_w1 = m->fire_packs[2000000 + pa];
      cc.fire_w3 = m->fire_packs[2000000 + pb];
      cc.fire_ws16 = nullptr;
      cc.fire_b1 = val(e1.in2).cptr;
      cc.fire_b3 = val(e3.in2).cptr;
      cc.flops_per_img = e1.flops_per_img + e3.flops_per_img;
      cc.bytes_per_img = 2.0 * double(e1.C * e1.H * e1.W) + 2.0 * double((e1.M + e3.M) * e1.H * e1.W);
      cc.name = e1.name.substr(0, e1.name.find('/')) + "/expand+concat";
      val(e1.out).elided = val(e3.out).elided = true;
      nop(e1); nop(e3);
    }
    recount();
    return ORE_OK;
  }

  // (7) the first conv + pool whose pooled map is read only by a small 1x1 conv (+ Relu) takes that
  // conv into its launch (SqueezeNet's conv1 + pool1 + fire2/squeeze1x1; the pooled map is never
  // stored).  Bit-identical to the separate squeeze (the same k-ordered chain over the same pooled
  // values).  f16: conv_pair_pool_f16_kernel SQ (<= 32 channels); f32: the window kernel (pooled-conv
  // variant 7, <= 16 channels).
  ore_status first_squeeze() {
    if (!has(ORE_FUSE_FIRST_SQUEEZE | ORE_FUSE_CONV_POOL | ORE_FUSE_CONV_RELU)) return ORE_OK;
    for (size_t i = 0; i < m->steps.size(); ++i) {
      Step& cv = st(int(i));
      if (cv.kind != S_CONV || !cv.epool || cv.c1sq || !private_value(cv.out)) continue;
      const bool f16 = cv.plan.f16 != 0;
      if (f16 ? (cv.plan.xmode != F16_X_NHWC_PAIR || cv.kh != 7 || cv.kw != 7 || cv.sh != 2 || cv.sw != 2 ||
                 cv.win.pl % 2 || cv.C > 4 || (cv.M != 64 && cv.M != 96))
              : (!cv.wc1 || cv.C != 3 || cv.M != 96))
        continue;
      const int qi = reader(cv.out, i + 1);
      if (qi < 0) continue;
      Step& q = st(qi);
      if (q.kind != S_CONV || !q.relu || q.pool || q.epool || q.kh != 1 || q.kw != 1 || q.sh != 1 || q.sw != 1 ||
          q.win.pt || q.win.pl || q.in0 != cv.out || q.C != cv.M || q.in2 < 0 || q.in1 < 0 || !val(q.in1).cptr)
        continue;
      if (f16 ? (!q.plan.f16 || q.plan.xmode != F16_X_NHWC_VEC || q.M > 32 || q.M % 8) : (q.plan.f16 || q.M > 16))
        continue;
      if (f16) {
        const int key = 5000000 + qi, M = int(q.M), C = int(q.C);
        const float* w = val(q.in1).cptr;
        if (!pack_once(key, fire_pack_f16_bytes(M, C, 1),
                       [&](float* buf) { launch_fire_pack_f16(w, M, C, 1, buf, m->ctx->stream); }))
          return err(m, ORE_ERR_HIP, "squeeze weight packing failed");
        cv.sq_w = m->fire_packs[key];
      } else {
        cv.sq_w = val(q.in1).cptr;  // ONNX [M][C][1][1] = [M][K]
        // untuned: the band walker for batches that give every CU an image (one workgroup per band of an
        // image; it bands smaller batches but the window kernel's patches fill the chip better there),
        // else the window kernel; an autotuned / set choice (epv 7 or 8) is kept
      }
      cv.c1sq = true;
      cv.sq_b = val(q.in2).cptr;
      cv.sq_M = q.M;
      if (!f16 && cv.plan.epv != EPOOL_BAND_VARIANT && cv.plan.epv != EPOOL_WIN_VARIANT)
        cv.plan.epv = m->max_batch >= 128 && band_step(cv) ? EPOOL_BAND_VARIANT : EPOOL_WIN_VARIANT;
      // f16: the band walker (one workgroup per image) for batches that give every CU an image, else the
      // patch kernel; an autotuned / set choice is kept
      if (f16 && cv.plan.epv != C1_BAND_F16_VARIANT && cv.plan.epv != C1_PATCH_F16_VARIANT)
        cv.plan.epv = m->max_batch >= 128 && band_f16_step(cv) ? C1_BAND_F16_VARIANT : C1_PATCH_F16_VARIANT;
      val(cv.out).elided = true;
      cv.out = q.out;
      cv.flops_per_img += q.flops_per_img;
      cv.bytes_per_img = double(val(cv.in0).es) * double(cv.C * cv.H * cv.W) + (f16 ? 2.0 : 4.0) * double(q.M * q.H * q.W);
      cv.name = cv.name + "+" + q.name;
      nop(q);
    }
    recount();
    return ORE_OK;
  }

  // (8) f32: a 3x3 / stride-2 MaxPool left standing (SqueezeNet pool5) whose only reader is a 1x1 Conv
  // (+ Relu) with <= 64 channels runs inside that conv (pool_conv1x1_f32_kernel, the pooled map never
  // stored).  Bit-identical to the MaxPool kernel + the conv.
  void pool_squeeze() {
    if (!has(ORE_FUSE_POOL_SQUEEZE) || m->f16) return;
    for (size_t i = 0; i < m->steps.size(); ++i) {
      Step& pl = st(int(i));
      if (pl.kind != S_MAXPOOL || pl.kh != 3 || pl.kw != 3 || pl.sh != 2 || pl.sw != 2) continue;
      const int v = pl.out;
      if (!private_value(v) || val(pl.in0).es != 4 || val(pl.in0).nhwc) continue;
      const int ci = reader(v, i + 1);
      if (ci < 0) continue;
      Step& cv = st(ci);
      if (cv.in0 != v || !pool_squeeze_fits(pl, cv)) continue;
      cv.pool = true;
      cv.in0 = pl.in0;
      cv.pH = pl.H; cv.pW = pl.W; cv.psh = pl.sh; cv.psw = pl.sw; cv.pwin = pl.win;
      cv.bytes_per_img = 4.0 * double(pl.C * pl.H * pl.W) + 4.0 * double(cv.M * cv.H * cv.W);
      cv.name = pl.name + "+" + cv.name;
      val(v).elided = true;
      nop(pl);
    }
    recount();
  }

  // (8a) f32: the pooled squeeze of (8) whose pool reads Concat(e1, e3), e1 a 1x1 conv + Relu of 32 / 64
  // channels read only by the Concat (SqueezeNet fire4 -> pool3 -> fire5, fire8 -> pool5 -> fire9 under
  // Winograd, wino_pool_split): e1 is recomputed inside pool_conv1x1_f32_kernel from its own input, so
  // its map (fire4: 128 x 54 x 54 floats per image) is neither written nor read back.  The Concat is
  // placed in memory here (e3 writes its slice; e1's slice is never materialised).  Bit-identical: the
  // same k-ordered MFMA chain, bias and Relu as the streaming 1x1 conv, the max of the same nine values.
  // Not under ORE_KEEP_VALUES (e1's output would not exist to read back).
  void pool_expand() {
    if (!has(ORE_FUSE_POOL_EXPAND | ORE_FUSE_POOL_SQUEEZE | ORE_FUSE_CONV_RELU | ORE_FUSE_CONCAT) ||
        has(ORE_KEEP_VALUES) || m->f16)
      return;
    for (size_t i = 0; i < m->steps.size(); ++i) {
      Step& cv = st(int(i));
      if (cv.kind != S_CONV || !cv.pool || cv.pe1 || cv.in0 < 0) continue;
      const int ci = producer[cv.in0];
      int pa, pb;
      if (ci < 0 || !fire_concat(ci, &pa, &pb)) continue;
      Step &cc = st(ci), &e1 = st(pa), &e3 = st(pb);
      // C1 = 64 (fire8 -> pool5) holds 48 B registers per lane and halves the launch's occupancy: 218 us
      // against 74 + 106 for the separate launches (profiles/r05_ab_pool_expand.txt), so 32 only unless eager
      if (!eager() && e1.C != 32) continue;
      if (!plain_1x1(e1) || e1.in2 < 0 || !e1.wp || (e1.C != 32 && e1.C != 64) || e1.M % 16 || e1.H != cv.pH ||
          e1.W != cv.pW || e3.kind != S_CONV || e3.epool || e3.pool)
        continue;
      // the Concat's only reader is this launch: e1's slice of it is never written
      if (!private_value(cc.in0) || !private_value(cc.in1) || !private_value(cc.out) || val(e1.in0).es != 4 ||
          val(e1.in0).nhwc || val(cc.in0).alias_of >= 0 || val(cc.in1).alias_of >= 0)
        continue;
      PoolConvParams q{};  // the kernel's limits with e1 inside
      q.C = int(cv.C); q.H = int(cv.pH); q.W = int(cv.pW); q.Hp = int(cv.pwin.Ho); q.Wp = int(cv.pwin.Wo);
      q.pt = int(cv.pwin.pt); q.pl = int(cv.pwin.pl); q.M = int(cv.M); q.Mp = cv.plan.Mp; q.Kp = cv.plan.krows;
      q.N = 1; q.x_ps = int(q.H * q.W); q.y_ps = int(q.Hp * q.Wp);
      q.x_nstride = int64_t(q.C) * q.x_ps; q.y_nstride = int64_t(q.M) * q.y_ps;
      q.s = q.w1 = q.b1 = e1.wp; q.C1 = int(e1.C); q.E1 = int(e1.M); q.w1_Mp = e1.plan.Mp; q.s_ps = q.H * q.W;
      if (!pool_conv1x1_f32_eligible(q)) continue;
      cv.pe1 = true;
      cv.in3 = e1.in0;
      cv.pe1_w = e1.wp;
      cv.pe1_b = val(e1.in2).cptr;
      cv.pe1_C = e1.C;
      cv.pe1_E = e1.M;
      cv.pe1_Mp = e1.plan.Mp;
      // work: e1 per band row it stages (2 PR + 1 input rows per PR pooled rows, neighbouring bands share one)
      const int pr = pool_conv1x1_f32_rows(int(cv.pwin.Wo));
      const double rows = double((cv.pwin.Ho + pr - 1) / pr * (2 * pr + 1));
      cv.mfma_flops_per_img = (cv.mfma_flops_per_img < 0 ? cv.flops_per_img : cv.mfma_flops_per_img) +
                              e1.flops_per_img * rows / double(e1.H);
      cv.flops_per_img += e1.flops_per_img;
      cv.bytes_per_img = 4.0 * double((cv.C - e1.M + e1.C) * cv.pH * cv.pW) + 4.0 * double(cv.M * cv.H * cv.W);
      cv.name = e1.name + "+" + cv.name;
      // Concat in place, e1's slice never written
      Value &a = val(cc.in0), &b = val(cc.in1);
      a.alias_of = cc.out; a.alias_ch = 0; a.slice = true; a.elided = true;
      b.alias_of = cc.out; b.alias_ch = a.dims[1]; b.slice = true;
      nop(cc);
      nop(e1);
    }
    recount();
  }

  // (8b) f16: a 1x1 conv (+ Relu) whose only reader is GlobalAveragePool runs with the GAP in its
  // epilogue (conv1x1_gap_f16_kernel: SqueezeNet conv10 -> relu10 -> pool10; the 87 MB map is never
  // stored).  Bit-identical to conv_f16 + gap_nhwc_kernel.  Not under ORE_KEEP_VALUES (the conv output
  // would not exist to read back).
  ore_status conv_gap() {
    if (!has(ORE_FUSE_CONV_GAP) || has(ORE_KEEP_VALUES)) return ORE_OK;
    for (size_t i = 0; i < m->steps.size(); ++i) {
      Step& g = st(int(i));
      if (g.kind != S_GAP) continue;
      const int v = g.in0;
      if (!m->f16) {  // f32: conv1x1_gap_f32_kernel (the conv's weights in launch_pack_cg_f32's layout)
        if (v < 0 || !private_value(v) || val(v).es != 4 || val(v).nhwc || producer[v] < 0) continue;
        Step& cv = st(producer[v]);
        if (cv.kind != S_CONV || cv.out != v || cv.plan.f16 || cv.plan.wino || cv.epool || cv.pool || cv.c1sq ||
            cv.kh != 1 || cv.kw != 1 || cv.sh != 1 || cv.sw != 1 || cv.win.pt != 0 || cv.win.pl != 0 ||
            cv.win.Ho != cv.H || cv.win.Wo != cv.W || cv.C % 32 != 0 || cv.H * cv.W > 256 || val(cv.in0).es != 4)
          continue;
        const int key = 4100000 + producer[v], M = int(cv.M), K = int(cv.C);
        const float* w = val(cv.in1).cptr;
        if (!pack_once(key, cg_f32_pack_bytes(M, K), [&](float* buf) { launch_pack_cg_f32(w, M, K, buf, m->ctx->stream); }))
          return err(m, ORE_ERR_HIP, "conv + GAP weight packing failed");
        cv.wc1 = m->fire_packs[key];
        cv.gap = true;
        cv.out = g.out;
        cv.bytes_per_img = 4.0 * double(cv.C * cv.H * cv.W) + 4.0 * double(cv.M);
        cv.name = cv.name + "+" + g.name;
        val(v).elided = true;
        nop(g);
        continue;
      }
      if (v < 0 || !private_value(v) || !val(v).nhwc || val(v).es != 2 || producer[v] < 0) continue;
      Step& cv = st(producer[v]);
      if (cv.kind != S_CONV || cv.out != v || !cv.plan.f16 || cv.plan.xmode != F16_X_NHWC_VEC || cv.epool || cv.pool ||
          cv.c1sq || cv.kh != 1 || cv.kw != 1 || cv.sh != 1 || cv.sw != 1 || cv.win.pt != 0 || cv.win.pl != 0 ||
          cv.win.Ho != cv.H || cv.win.Wo != cv.W || cv.C % 64 != 0 || cv.H * cv.W > 256)
        continue;
      cv.gap = true;
      cv.out = g.out;
      cv.bytes_per_img = 2.0 * double(cv.C * cv.H * cv.W) + 4.0 * double(cv.M);
      cv.name = cv.name + "+" + g.name;
      val(v).elided = true;
      nop(g);
    }
    recount();
    return ORE_OK;
  }

  // (9) algorithm selection, a load-time rule (never by timing): f32 models with Winograd on run every
  // 3x3 / stride-1 / pad-1 conv not taken by a direct-kernel fusion by Winograd F(2x2, 3x3)
  void select_algorithms() {
    for (auto& s : m->steps) {
      if (m->wino && s.kind == S_CONV && s.has_wino && !s.pool && !s.epool) {
        s.plan = s.plan_wino;
        s.wp = s.wp_wino;
        s.ktab = nullptr;
        // MFMA work issued: 16 positions x C x M per 2x2 output tile (the direct conv's 36 C M / 4 pixels)
        s.mfma_flops_per_img = 2.0 * 16.0 * double(s.C) * double(s.M) * double((s.win.Ho + 1) / 2) *
                               double((s.win.Wo + 1) / 2);
      }
    }
  }

  // (10) Dropout / activation Reshape as aliases
  void alias_copies() {
    if (!has(ORE_FUSE_ALIAS)) return;
    for (auto& s : m->steps) {
      if (s.kind != S_COPY) continue;
      val(s.out).alias_of = s.in0;  // resolved to the root at run time; requires a contiguous source
      s.kind = S_NOP;
    }
  }

  // (11) Concat in place: producers write channel slices of the concat buffer
  void concat_in_place() {
    if (!has(ORE_FUSE_CONCAT)) return;
    for (auto& s : m->steps) {
      if (s.kind != S_CONCAT || s.axis != 1 || s.in0 == s.in1) continue;
      Value &a = val(s.in0), &b = val(s.in1);
      const int pa = producer[s.in0], pb = producer[s.in1];
      if (pa < 0 || pb < 0 || !strided_writer(st(pa)) || !strided_writer(st(pb))) continue;
      if (a.uses != 1 || b.uses != 1 || a.is_output || b.is_output || a.alias_of >= 0 || b.alias_of >= 0) continue;
      a.alias_of = s.out; a.alias_ch = 0; a.slice = true;
      b.alias_of = s.out; b.alias_ch = a.dims[1]; b.slice = true;
      s.kind = S_NOP;
    }
  }

  int root(int id) const {
    while (m->values[id].alias_of >= 0) id = m->values[id].alias_of;
    return id;
  }

  // (12) layout: an activation touched only by Conv / MaxPool kernels (and f32 GlobalAveragePool)
  // gets channel planes padded to a multiple of 32 floats (128-B aligned rows for the conv epilogue
  // and the 1x1 gathers) when that costs <= 5 % extra columns; everything else stays dense NCHW.
  ore_status layout_planes() {
    for (auto& v : m->values) {  // aliases of aliases must stay contiguous views (Reshape / Dropout of a slice)
      if (v.alias_of < 0 || v.slice) continue;
      if (val(v.alias_of).slice) return err(m, ORE_ERR_INVALID, "internal: alias of a strided view (" + v.name + ")");
    }
    std::vector<char> dense(m->values.size(), 0);
    for (const Step& s : m->steps) {
      if (s.kind == S_NOP) continue;
      const bool ok = s.kind == S_CONV || s.kind == S_FIRE || s.kind == S_MAXPOOL || (s.kind == S_GAP && !val(s.in0).nhwc);
      for (int id : {s.in0, s.in2, s.in3, s.out})
        if (id >= 0 && !val(id).is_const && !ok) dense[root(id)] = 1;
      if (s.in1 >= 0 && !val(s.in1).is_const) dense[root(s.in1)] = 1;
    }
    // a contiguous view (Dropout / Reshape alias) keeps its root's planes only as a 4-D
    // intermediate; as a graph output or a reshaped 2-D value it needs the dense layout
    for (size_t id = 0; id < m->values.size(); ++id) {
      const Value& v = m->values[id];
      if (v.alias_of >= 0 && !v.slice && (v.is_output || v.ndim != 4)) dense[root(int(id))] = 1;
    }
    for (size_t id = 0; id < m->values.size(); ++id) {
      Value& v = m->values[id];
      if (v.is_const || v.ndim != 4 || v.alias_of >= 0) continue;
      if (v.nhwc) {  // channels-last f16: dense pixels of dims[1] channels
        v.ps = v.dims[1];
        continue;
      }
      const int64_t P = v.dims[2] * v.dims[3];
      const bool pad = has(ORE_FUSE_CONCAT) && !dense[id] && !v.is_input && !v.is_output;
      v.ps = pad ? padded_plane(P) : P;
    }
    for (size_t id = 0; id < m->values.size(); ++id) {  // views inherit the plane stride of their root
      Value& v = m->values[id];
      if (v.alias_of < 0 || v.ndim != 4) continue;
      const Value& r = val(root(int(id)));
      v.ps = r.ps;
      if (v.nhwc != r.nhwc) return err(m, ORE_ERR_INVALID, "internal: view of a different layout (" + v.name + ")");
      if (!v.slice && r.ps != (r.nhwc ? r.dims[1] : r.dims[2] * r.dims[3]) &&
          (v.is_output || v.dims[2] * v.dims[3] != r.dims[2] * r.dims[3]))
        return err(m, ORE_ERR_INVALID, "internal: dense alias of a padded value (" + v.name + ")");
    }
    return ORE_OK;
  }

  // (13) one device arena: every materialised root value gets a slot sized for run_batch, slots reused
  // by liveness (first fit over [first write, last read] intervals)
  ore_status assign_arena() {
    const int nsteps = int(m->steps.size());
    for (int i = 0; i < nsteps; ++i) {
      const Step& s = m->steps[i];
      if (s.kind == S_NOP) continue;
      for (int id : {s.in0, s.in1, s.in2, s.in3}) {
        if (id < 0 || val(id).is_const) continue;
        Value& r = val(root(id));
        if (r.first < 0) r.first = i;
        r.last = std::max(r.last, i);
      }
      if (s.out >= 0) {
        Value& r = val(root(s.out));
        if (r.first < 0 || r.first > i) r.first = i;
        r.last = std::max(r.last, i);
      }
    }
    // the model output stays live to the end (it may be copied out after the last step)
    if (m->output_value >= 0) val(root(m->output_value)).last = nsteps;

    struct Slot { int64_t off, size; int first, last; };
    std::vector<int> roots;
    for (size_t id = 0; id < m->values.size(); ++id) {
      const Value& v = m->values[id];
      if (v.is_const || v.is_input || v.alias_of >= 0 || v.elided || v.first < 0) continue;
      roots.push_back(int(id));
    }
    // the kernels address a launch's activations through buffer resources and 32-bit offsets: one pass
    // of the graph covers run_batch images, the largest batch whose every value (the caller's input and
    // output included) and the f16 input conversion stay below RUN_LIMIT bytes; ore_model_run runs
    // larger batches in image chunks (config 4's 2048 images per GPU: fire4's concat is 3 MB per image)
    constexpr int64_t RUN_LIMIT = (int64_t(1) << 31) - (int64_t(1) << 21);
    int64_t per_img_max = 0;
    for (size_t id = 0; id < m->values.size(); ++id) {
      const Value& v = m->values[id];
      if (v.is_const || v.alias_of >= 0 || v.elided || (v.first < 0 && !v.is_input)) continue;
      per_img_max = std::max(per_img_max, v.image_stride() * v.es);
    }
    int64_t xcvt_img = 0;
    for (const Step& s : m->steps)
      if (s.kind == S_CONV && s.plan.f16 && s.plan.xmode == F16_X_NHWC_PAIR) xcvt_img = std::max(xcvt_img, s.H * s.W * 4 * 2);
    per_img_max = std::max(per_img_max, xcvt_img);
    if (per_img_max >= RUN_LIMIT) return err(m, ORE_ERR_UNSUPPORTED, "one image's activations exceed 2 GiB");
    m->run_batch = std::min<int64_t>(m->max_batch, per_img_max > 0 ? RUN_LIMIT / per_img_max : m->max_batch);
    if (xcvt_img && size_t(xcvt_img * m->run_batch) > m->xcvt_bytes) {
      if (m->xcvt) (void)hipFree(m->xcvt);
      m->xcvt = nullptr;
      m->xcvt_bytes = 0;
      if (hipMalloc(&m->xcvt, size_t(xcvt_img * m->run_batch)) != hipSuccess)
        return err(m, ORE_ERR_OOM, "input conversion buffer allocation failed");
      m->xcvt_bytes = size_t(xcvt_img * m->run_batch);
    }
    std::sort(roots.begin(), roots.end(), [&](int a, int b) { return val(a).image_stride() > val(b).image_stride(); });
    std::vector<Slot> placed;
    int64_t arena = 0;
    for (int id : roots) {
      Value& v = val(id);
      const int64_t size = ((v.image_stride() * m->run_batch * v.es) + 255) / 256 * 256;
      std::vector<std::pair<int64_t, int64_t>> busy;  // slots whose lifetimes overlap this one
      for (auto& s : placed)
        if (has(ORE_KEEP_VALUES) || !(s.last < v.first || v.last < s.first)) busy.push_back({s.off, s.off + s.size});
      std::sort(busy.begin(), busy.end());
      int64_t off = 0;
      for (auto& b : busy) {
        if (off + size <= b.first) break;
        off = std::max(off, b.second);
      }
      v.arena_off = off;
      placed.push_back({off, size, v.first, v.last});
      arena = std::max(arena, off + size);
    }
    if (size_t(arena) > m->arena_bytes) {
      if (m->arena_alloc) (void)hipFree(m->arena_alloc);
      m->arena = m->arena_alloc = nullptr;
      m->arena_bytes = 0;
      if (arena > 0 && hipMalloc(reinterpret_cast<void**>(&m->arena_alloc), size_t(arena) + 4096) != hipSuccess)
        return err(m, ORE_ERR_OOM, "arena allocation of " + std::to_string(arena) + " bytes failed");
      if (m->arena_alloc) m->arena = m->arena_alloc + 4096;
      m->arena_bytes = size_t(arena);
    }
    m->exec_steps.clear();
    for (int i = 0; i < nsteps; ++i)
      if (m->steps[i].kind != S_NOP) m->exec_steps.push_back(i);
    return ORE_OK;
  }

  // (14) independent neighbours for the two-stream issue (ore_model_set_streams): B reads nothing A
  // writes, and no byte range A or B writes overlaps one the other reads or writes (arena slots are
  // shared by liveness, so check the memory)
  void pair_steps() {
    m->pair_next.assign(m->exec_steps.size(), 0);
    auto span = [&](int id, int64_t* lo, int64_t* hi) {  // arena byte range of a value's root
      const Value& v = val(root(id));
      if (v.is_const || v.arena_off < 0) return false;
      *lo = v.arena_off;
      *hi = v.arena_off + v.image_stride() * m->run_batch * v.es;
      return true;
    };
    auto overlap = [&](int a, int b) {
      if (a < 0 || b < 0 || val(a).is_const || val(b).is_const) return false;
      const int ra = root(a), rb = root(b);
      if (val(ra).is_input || val(rb).is_input) return false;  // never written
      if (ra == rb) {  // channel slices of one buffer: disjoint unless the same slice
        const Value &va = val(a), &vb = val(b);
        if (va.slice && vb.slice) return va.alias_ch < vb.alias_ch + vb.dims[1] && vb.alias_ch < va.alias_ch + va.dims[1];
        return true;
      }
      if (val(ra).is_output || val(rb).is_output) return true;  // conservative (may live in the arena)
      int64_t a0, a1, b0, b1;
      if (!span(a, &a0, &a1) || !span(b, &b0, &b1)) return false;
      return a0 < b1 && b0 < a1;
    };
    for (size_t k = 0; k + 1 < m->exec_steps.size(); ++k) {
      if (k > 0 && m->pair_next[k - 1]) continue;  // pairs only
      const Step &A = st(m->exec_steps[k]), &B = st(m->exec_steps[k + 1]);
      bool ok = A.out >= 0 && B.out >= 0;
      for (int bi : {B.in0, B.in1, B.in2, B.in3}) ok = ok && !overlap(bi, A.out);
      for (int ai : {A.in0, A.in1, A.in2, A.in3}) ok = ok && !overlap(ai, B.out);
      ok = ok && !overlap(A.out, B.out);
      m->pair_next[k] = ok ? 1 : 0;
    }
  }

  // (15) gather tables: they depend on the input's plane stride
  ore_status gather_tables() {
    for (const Step& s : m->steps) {
      if (s.kind != S_CONV || !s.ktab) continue;
      const Value& xv = val(s.in0);
      int2* kt = const_cast<int2*>(s.ktab);
      if (s.plan.f16 && s.plan.xmode != F16_X_NCHW32)
        launch_ktab_nhwc(kt, s.plan.xmode, int(s.C), int(s.kh), int(s.kw),
                         s.plan.xmode == F16_X_NHWC_PAIR ? 4 : int(xv.ps), int(s.W), m->ctx->stream);
      else
        launch_ktab(kt, int(s.C * s.kh * s.kw), int(s.kh), int(s.kw), int(xv.ps ? xv.ps : s.H * s.W), int(s.W),
                    m->ctx->stream);
    }
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(m->ctx->stream) != hipSuccess)
      return err(m, ORE_ERR_HIP, "gather table build failed");
    return ORE_OK;
  }
};

ore_status plan(ore_model* m) {
  m->steps = m->base_steps;
  if (!m->n_base_values) m->n_base_values = m->values.size();
  m->values.resize(m->n_base_values);  // drop the previous plan's views
  for (auto& v : m->values) {
    v.alias_of = -1; v.alias_ch = 0; v.slice = false; v.ps = 0; v.elided = false; v.arena_off = -1;
    v.nhwc = !v.is_const && v.es == 2 && v.ndim == 4;
    v.first = v.last = -1;
  }
  count_uses(m, m->steps);
  Planner p{m, std::vector<int>(m->values.size(), -1)};
  for (size_t i = 0; i < m->steps.size(); ++i)
    if (m->steps[i].out >= 0 && m->steps[i].kind != S_NOP) p.producer[m->steps[i].out] = int(i);
  p.conv_relu();
  if (ore_status st = p.conv_pool()) return st;
  if (ore_status st = p.fire_pool_f32()) return st;
  p.concat_pool();
  if (ore_status st = p.fire_f32()) return st;
  if (ore_status st = p.fire_f16()) return st;
  if (ore_status st = p.fire_f16_concat()) return st;
  if (ore_status st = p.first_squeeze()) return st;
  p.pool_squeeze();
  p.pool_expand();
  if (ore_status st = p.conv_gap()) return st;
  p.select_algorithms();
  p.alias_copies();
  p.concat_in_place();
  if (ore_status st = p.layout_planes()) return st;
  if (ore_status st = p.assign_arena()) return st;
  p.pair_steps();
  return p.gather_tables();
}

// storage of a value for the current run: pointer to image 0 and per-image stride
struct Ref { float* p; int64_t nstride; int64_t ps; int es; };  // p: storage of es-byte elements

Ref ref_of(ore_model* m, int id) {
  const Value& v = m->values[id];
  if (v.is_const) return {v.cptr, 0, 0, 4};
  if (v.alias_of >= 0) {
    Ref base = ref_of(m, v.alias_of);
    if (v.slice)  // NCHW: the slice's first plane; NHWC: its first channel inside each pixel
      return {reinterpret_cast<float*>(reinterpret_cast<char*>(base.p) + v.alias_ch * (v.nhwc ? 1 : base.ps) * base.es),
              base.nstride, base.ps, base.es};
    return base;
  }
  if (v.is_input) return {const_cast<float*>(m->cur_in), v.image_stride(), v.ps, v.es};
  if (v.is_output && m->out_bound) return {m->cur_out, v.image_stride(), v.ps, v.es};
  return {reinterpret_cast<float*>(m->arena + v.arena_off), v.image_stride(), v.ps, v.es};
}

// steps on NHWC f16 values (f16 models): Relu, GAP (f32 out), Concat (channels), Dropout copies
ore_status launch_step_f16(ore_model* m, const Step& s, int64_t n) {
  ore_ctx* ctx = m->ctx;
  const Value& X = m->values[s.in0];
  const Ref x = ref_of(m, s.in0), y = ref_of(m, s.out);
  const int64_t count = n * X.per_image();
  if (count == 0) return ORE_OK;
  if (s.kind == S_GAP) {
    launch_gap_nhwc(x.p, reinterpret_cast<float*>(y.p), int(n), int(X.dims[1]), int(X.dims[2] * X.dims[3]), int(x.ps),
                    x.nstride, ctx->stream);
    ORE_HIP_CHECK(ctx, hipGetLastError());
    return ORE_OK;
  }
  if (x.nstride != X.per_image() || y.nstride != m->values[s.out].per_image())
    return err(m, ORE_ERR_INVALID, "internal: f16 step on a strided view");
  switch (s.kind) {
    case S_RELU: launch_relu_f16(x.p, y.p, count, ctx->stream); break;
    case S_COPY:
      if (x.p != y.p)
        ORE_HIP_CHECK(ctx, hipMemcpyAsync(y.p, x.p, size_t(count) * 2, hipMemcpyDeviceToDevice, ctx->stream));
      break;
    case S_CONCAT: {  // axis 1 (build_node): per pixel, a's channels then b's
      const Value& B = m->values[s.in1];
      const Ref b = ref_of(m, s.in1);
      if (b.nstride != B.per_image() || s.axis != 1)
        return err(m, ORE_ERR_INVALID, "internal: f16 concat of a strided view");
      launch_concat_nhwc(x.p, b.p, y.p, n * X.dims[2] * X.dims[3], int(X.dims[1]), int(B.dims[1]), ctx->stream);
      break;
    }
    default: return err(m, ORE_ERR_UNSUPPORTED, "internal: step '" + s.name + "' has no f16 kernel");
  }
  ORE_HIP_CHECK(ctx, hipGetLastError());
  return ORE_OK;
}

ore_status launch_step(ore_model* m, const Step& s, int64_t n) {
  ore_ctx* ctx = m->ctx;
  const Ref y = ref_of(m, s.out);
  switch (s.kind) {
    case S_CONV: {
      const Ref x = ref_of(m, s.in0);
      const float* bias = s.in2 >= 0 ? m->values[s.in2].cptr : nullptr;
      const F16Epool ep{s.ep_kh, s.ep_kw, s.ep_sh, s.ep_sw, s.ep_win};
      // the one-launch f16 first conv + pool from the f32 input (plan.epv 1: the two-launch patch path)
      if (s.plan.f16 && s.plan.xmode == F16_X_NHWC_PAIR && s.epool && (s.c1sq || s.plan.epv != 1)) {
        bool ran = false;
        const C1Squeeze sq{s.sq_w, s.sq_b, int(s.sq_M), y.p, y.nstride, int(y.ps ? y.ps : s.sq_M)};
        const ore_status st = run_conv_pair_pool_f16(ctx, s.plan, x.p, n, s.C, s.H, s.W, x.nstride, x.ps, s.wp, s.M, s.kh,
                                                     s.kw, bias, s.win, s.sh, s.sw, s.relu, s.c1sq ? nullptr : y.p,
                                                     y.nstride, s.c1sq ? s.M : y.ps, ep, &ran, s.c1sq ? &sq : nullptr);
        if (ran) s.ran_tile = last_conv_tile;  // C1_POOL_F16_TILE or C1_BAND_F16_TILE
        if (st != ORE_OK || ran) return st;
        s.ran_tile = -1;
        if (s.c1sq) return err(m, ORE_ERR_INVALID, "internal: the fused first conv + squeeze declined its launch");
      }
      if (s.plan.f16 && s.plan.xmode == F16_X_NHWC_PAIR) {
        // convert the f32 NCHW input to NHWC f16 (4 channels per pixel), then gather
        const int cs = 4;
        launch_nchw_to_nhwc(x.p, m->xcvt, int(n), int(s.C), int(s.H * s.W), x.nstride, int(x.ps ? x.ps : s.H * s.W), cs,
                            ctx->stream);
        ORE_HIP_CHECK(ctx, hipGetLastError());
        const ore_status r = run_conv_f16(ctx, s.plan, m->xcvt, n, s.C, s.H, s.W, s.H * s.W * cs, cs, s.wp, s.ktab, s.M,
                                          s.kh, s.kw, bias, s.win, s.sh, s.sw, s.relu, y.p, y.nstride, y.ps,
                                          s.epool ? &ep : nullptr);
        if (s.epool) s.ran_tile = last_conv_tile = EPOOL_TILE_BASE + 1;  // "epool patch": conv_f16's pooled epilogue
        return r;
      }
      if (s.plan.f16 && s.gap) {
        const Conv1x1GapF16 q{x.p, s.wp, bias, y.p, int(n), int(s.C), int(s.H * s.W), int(s.M), s.plan.Mp,
                              int((s.C + 31) / 32 * 32), int(x.ps), s.relu ? 1 : 0, x.nstride, y.nstride};
        if (!conv1x1_gap_f16_eligible(q)) return err(m, ORE_ERR_INVALID, "internal: conv + GAP on an unsupported layout");
        launch_conv1x1_gap_f16(q, ctx->stream);
        ORE_HIP_CHECK(ctx, hipGetLastError());
        s.ran_tile = last_conv_tile = CONV_GAP_F16_TILE;
        return ORE_OK;
      }
      if (s.gap) {  // f32: conv1x1_gap_f32_kernel
        const Conv1x1GapF32 q{x.p, s.wc1, bias, y.p, int(n), int(s.C), int(s.H * s.W), int(s.M),
                              int(x.ps ? x.ps : s.H * s.W), s.relu ? 1 : 0, x.nstride, y.nstride};
        if (!conv1x1_gap_f32_eligible(q)) return err(m, ORE_ERR_INVALID, "internal: conv + GAP on an unsupported layout");
        if (n > 0) launch_conv1x1_gap_f32(q, ctx->stream);
        ORE_HIP_CHECK(ctx, hipGetLastError());
        s.ran_tile = last_conv_tile = CONV_GAP_F32_TILE;
        return ORE_OK;
      }
      if (s.plan.f16)
        return run_conv_f16(ctx, s.plan, x.p, n, s.C, s.H, s.W, x.nstride, x.ps, s.wp, s.ktab, s.M, s.kh, s.kw, bias,
                            s.win, s.sh, s.sw, s.relu, y.p, y.nstride, y.ps, s.epool ? &ep : nullptr);
      if (s.epool) {
        ctx->mapped_lo = m->arena_alloc;  // the arena and its 4 KiB lead are mapped
        ctx->mapped_hi = m->arena ? m->arena + m->arena_bytes : nullptr;
        const int64_t pplane = s.ep_win.Ho * s.ep_win.Wo;
        const C1SqueezeF32 sq1{static_cast<const float*>(s.sq_w), s.sq_b, int(s.sq_M), y.p, y.nstride,
                               int(y.ps ? y.ps : pplane)};
        const ore_status r = run_conv_epool(ctx, s.plan, x.p, n, s.C, s.H, s.W, x.nstride, x.ps, s.wp, s.ktab, s.M, s.kh,
                                            s.kw, bias, s.win, s.sh, s.sw, s.relu, s.ep_kh, s.ep_kw, s.ep_sh, s.ep_sw,
                                            s.ep_win, s.c1sq ? nullptr : y.p, y.nstride, s.c1sq ? pplane : y.ps, s.wc1,
                                            s.c1sq ? &sq1 : nullptr);
        ctx->mapped_lo = ctx->mapped_hi = nullptr;
        s.ran_tile = last_conv_tile;
        return r;
      }
      if (s.pool) {
        PoolExpand pe{};
        if (s.pe1) {
          const Ref sv = ref_of(m, s.in3);
          pe = {sv.p, s.pe1_w, s.pe1_b, int(s.pe1_C), int(s.pe1_E), s.pe1_Mp,
                sv.ps ? sv.ps : s.pH * s.pW, sv.nstride};
        }
        return run_conv_pool(ctx, s.plan, x.p, n, s.C, s.pH, s.pW, x.nstride, x.ps, s.pwin, s.psh, s.psw, s.wp, s.M, bias,
                             s.relu, y.p, y.nstride, y.ps, x.es, s.pe1 ? &pe : nullptr);
      }
      ctx->mapped_lo = m->arena_alloc;  // the arena and its 4 KiB lead are mapped
      ctx->mapped_hi = m->arena ? m->arena + m->arena_bytes : nullptr;
      const ore_status st = run_conv(ctx, s.plan, x.p, n, s.C, s.H, s.W, x.nstride, s.wp, s.ktab, s.M, s.kh, s.kw, bias,
                                     s.win, s.sh, s.sw, s.relu, y.p, y.nstride, x.ps, y.ps, x.es);
      ctx->mapped_lo = ctx->mapped_hi = nullptr;
      return st;
    }
    case S_FIRE: {
      const Ref x = ref_of(m, s.in0);
      if (s.fire_f16)
        return run_fire_f16(ctx, x.p, n, s.fire_C, s.fire_pool ? s.fire_H : s.H, s.fire_pool ? s.fire_W : s.W,
                            x.nstride, x.ps ? x.ps : s.fire_C, s.fire_w1, s.fire_b1, s.fire_E1, s.fire_w3, s.fire_b3,
                            s.fire_E3, s.fire_ws16, s.in2 >= 0 ? m->values[s.in2].cptr : nullptr, s.M, y.p,
                            y.nstride, y.ps ? y.ps : (s.M ? s.M : s.fire_E1 + s.fire_E3),
                            s.fire_pool ? &s.fire_pwin : nullptr);
      ctx->mapped_lo = m->arena_alloc;  // the arena and its 4 KiB lead are mapped
      ctx->mapped_hi = m->arena ? m->arena + m->arena_bytes : nullptr;
      const int64_t fH = s.fire_pool ? s.fire_H : s.H, fW = s.fire_pool ? s.fire_W : s.W;
      const ore_status st = run_fire(ctx, x.p, n, s.fire_C, fH, fW, x.nstride, x.ps ? x.ps : fH * fW, s.fire_w1,
                                     s.fire_b1, s.fire_E1, s.fire_w3, s.fire_b3, s.fire_E3, s.wp, s.plan.Mp,
                                     m->values[s.in2].cptr, s.M, y.p, y.nstride, y.ps ? y.ps : s.H * s.W,
                                     s.fire_pool ? &s.fire_pwin : nullptr);
      ctx->mapped_lo = ctx->mapped_hi = nullptr;
      return st;
    }
    case S_MATMUL: {
      const Ref x = ref_of(m, s.in0);
      return run_conv(ctx, s.plan, x.p, n, s.C, 1, 1, x.nstride, s.wp, s.ktab, s.M, 1, 1, nullptr, s.win, 1, 1, false, y.p,
                      y.nstride);
    }
    case S_MAXPOOL: {
      const Ref x = ref_of(m, s.in0);
      if (x.es == 2)
        return run_maxpool_nhwc(ctx, x.p, n, s.C, s.H, s.W, x.nstride, x.ps, s.kh, s.kw, s.win, s.sh, s.sw, y.p,
                                y.nstride, y.ps);
      return run_maxpool(ctx, x.p, n, s.C, s.H, s.W, x.nstride, s.kh, s.kw, s.win, s.sh, s.sw, y.p, y.nstride, x.ps,
                         y.ps, x.es);
    }
    default: break;
  }
  if (s.kind == S_GAP && m->values[s.in0].es == 4) {  // f32 NCHW rows, possibly padded planes
    const Value& X = m->values[s.in0];
    const Ref x = ref_of(m, s.in0);
    const int64_t HW = X.dims[2] * X.dims[3], ps = x.ps ? x.ps : HW;
    if (x.nstride != X.dims[1] * ps || y.nstride != X.dims[1])
      return err(m, ORE_ERR_INVALID, "internal: GlobalAveragePool on a strided view");
    launch_gap(x.p, 4, y.p, n * X.dims[1], int(HW), int(ps), ctx->stream);
    ORE_HIP_CHECK(ctx, hipGetLastError());
    return ORE_OK;
  }
  if (m->values[s.in0].es == 2) return launch_step_f16(m, s, n);
  // contiguous ops through the public entry points
  auto as_tensor = [&](int id, int64_t batch) {
    const Value& v = m->values[id];
    const Ref r = ref_of(m, id);
    ore_tensor t{};
    t.data = r.p;
    t.ndim = v.ndim;
    for (int i = 0; i < v.ndim; ++i) t.dims[i] = v.dims[i];
    if (!v.is_const) t.dims[0] = batch;
    t.nstride = v.is_const ? 0 : r.nstride;
    return t;
  };
  ore_tensor X = as_tensor(s.in0, n), Y = as_tensor(s.out, n);
  switch (s.kind) {
    case S_RELU: return ore_relu_f32(ctx, &X, &Y);
    case S_SOFTMAX: return ore_softmax_f32(ctx, &X, &Y);
    case S_GAP: return ore_gap_f32(ctx, &X, &Y);
    case S_COPY: return ore_dropout_f32(ctx, &X, &Y);
    case S_ADD: {
      ore_tensor B = as_tensor(s.in1, n);
      return ore_add_f32(ctx, &X, &B, &Y);
    }
    case S_CONCAT: {
      ore_tensor B = as_tensor(s.in1, n);
      return ore_concat_f32(ctx, &X, &B, s.axis, &Y);
    }
    default: return err(m, ORE_ERR_INVALID, "internal: unexpected step kind");
  }
}

}  // namespace

namespace {

// the tile ids a step may run (its kernel family): autotune candidates and ore_model_set_step_tile's
// accepted values; empty for steps with one fixed kernel
// the band walker's geometry for a fused f32 first conv + pool + squeeze step (its layout checks are the
// launch's: a layout it declines runs the window kernel)
bool band_f16_step(const Step& s) {
  return s.plan.f16 && conv_band_pool_f16_geometry(int(s.C), int(s.M), int(s.kh), int(s.kw), int(s.sh), int(s.sw),
                                                   int(s.win.pt), int(s.win.pl), int(s.W), int(s.win.Wo),
                                                   int(s.ep_win.Ho), int(s.ep_win.Wo), int(s.ep_win.pt), int(s.ep_win.pl),
                                                   int(s.sq_M)) &&
         s.relu;
}

bool band_step(const Step& s) {
  return conv_band_pool_f32_geometry(int(s.C), int(s.M), int(s.kh), int(s.kw), int(s.sh), int(s.sw), int(s.win.pt),
                                     int(s.win.pl), int(s.W), int(s.win.Wo), int(s.ep_win.Ho), int(s.ep_win.Wo),
                                     int(s.ep_win.pt), int(s.ep_win.pl), int(s.sq_M), s.relu);
}

std::vector<int> step_tile_family(const Step& s) {
  std::vector<int> c;
  if (s.kind != S_CONV && s.kind != S_MATMUL) return c;
  if (s.kind == S_CONV && s.epool && !s.plan.f16) {  // f32 pooled conv: patch / row-walk variants, the window kernel
    if (s.c1sq) {  // the fused squeeze: window kernel, band walker (where its geometry allows it)
      if (band_step(s)) return {EPOOL_WIN_TILE, EPOOL_BAND_TILE};
      return {EPOOL_WIN_TILE};
    }
    for (int v = 1; v <= 5; ++v) c.push_back(EPOOL_TILE_BASE + v);
    if (s.wc1) c.push_back(EPOOL_WIN_TILE);
    return c;
  }
  if (s.kind == S_CONV && s.epool && s.plan.f16 && s.plan.xmode == F16_X_NHWC_PAIR) {  // f16 first conv + pool
    if (s.c1sq) {  // the fused squeeze: the patch kernel, the band walker (where its geometry allows it)
      if (band_f16_step(s)) return {C1_POOL_F16_TILE, C1_BAND_F16_TILE};
      return {C1_POOL_F16_TILE};
    }
    return {EPOOL_TILE_BASE + 1, C1_POOL_F16_TILE};  // two launches (conversion + patch kernel) / one launch
  }
  if (s.epool || s.pool || s.gap) return c;  // other f16 pooled epilogues / the pooled 1x1 / conv + GAP: one kernel
  if (s.plan.wino) {
    for (int t = 0; t < WINO_TILES_N; ++t) c.push_back(WINO_TILE_BASE + t);
    return c;
  }
  for (int t = 0; t < 4; ++t) c.push_back(t);  // the LDS-staged conv_gemm tiles
  // the LDS-free streaming kernel (f32 convs; launch_conv falls back to tile 0 where the geometry does
  // not allow it)
  if (!s.plan.f16 && s.kind == S_CONV)
    for (int t = CONV_TILE_STREAM; t < CONV_TILES_F32; ++t) c.push_back(t);
  if (!s.plan.f16 && s.kind == S_CONV && s.kh == 1 && s.kw == 1)  // the persistent 1x1 tiles
    for (int t = CONV_TILE_SP; t < CONV_TILE_SP + CONV_TILES_SP; ++t) c.push_back(t);
  return c;
}

// writes tile t into the step's plan (and the base step the next plan() copies from)
void set_tile(ore_model* m, int k, int t) {
  Step& s = m->steps[m->exec_steps[k]];
  Step& b = m->base_steps[m->exec_steps[k]];
  if (s.kind == S_CONV && s.epool) {
    const int v = t == EPOOL_WIN_TILE    ? EPOOL_WIN_VARIANT
                  : t == EPOOL_BAND_TILE ? EPOOL_BAND_VARIANT
                  : t == C1_POOL_F16_TILE ? (s.c1sq ? C1_PATCH_F16_VARIANT : 0)
                  : t == C1_BAND_F16_TILE ? C1_BAND_F16_VARIANT
                                          : t - EPOOL_TILE_BASE;
    s.plan.epv = b.plan.epv = v;
    return;
  }
  s.plan.cfg = t;
  if (s.plan.wino) b.plan_wino.cfg = t;
  else b.plan.cfg = t;
}

}  // namespace

extern "C" {

ore_status ore_model_load(ore_ctx* ctx, const void* bytes, size_t len, int64_t max_batch, ore_model** out) {
  return ore_model_load_ex(ctx, bytes, len, max_batch, 0, out);
}

ore_status ore_model_parse(const void* bytes, size_t len) {
  if (!bytes) return set_error(nullptr, ORE_ERR_INVALID, "null argument");
  Graph g;
  std::string perr;
  if (!parse_model(static_cast<const uint8_t*>(bytes), len, &g, &perr)) return set_error(nullptr, ORE_ERR_PARSE, "%s", perr.c_str());
  return ORE_OK;
}

ore_status ore_model_load_ex(ore_ctx* ctx, const void* bytes, size_t len, int64_t max_batch, int32_t flags,
                             ore_model** out) {
  if (!ctx || !bytes || !out || max_batch <= 0) return set_error(ctx, ORE_ERR_INVALID, "invalid argument");
  if (flags & ORE_LOAD_RETIRED_MASK)
    return set_error(ctx, ORE_ERR_UNSUPPORTED, "load flags 0x%x were retired in ABI 2 (the bf16x3 kernels, ORE_LOAD_X3)",
                     unsigned(flags & ORE_LOAD_RETIRED_MASK));
  if (flags & ~(ORE_LOAD_F16 | ORE_LOAD_NO_WINOGRAD))
    return set_error(ctx, ORE_ERR_INVALID, "unknown load flags 0x%x", unsigned(flags));
  ORE_HIP_CHECK(ctx, hipSetDevice(ctx->device));
  Graph g;
  std::string perr;
  if (!parse_model(static_cast<const uint8_t*>(bytes), len, &g, &perr)) return set_error(ctx, ORE_ERR_PARSE, "%s", perr.c_str());
  ore_model* m = new ore_model();
  m->ctx = ctx;
  m->max_batch = max_batch;
  m->f16 = (flags & ORE_LOAD_F16) != 0;
  m->wino = !m->f16 && (flags & ORE_LOAD_NO_WINOGRAD) == 0;
  m->conv_tile = ctx->conv_tile;
  auto fail = [&](ore_status st) {
    ore_model_destroy(m);
    return st;
  };
  // initializers: shapes from graph.input when listed there (get_input_data_shape, utils.rs:53-97),
  // else TensorProto.dims; f32 data uploaded once into one allocation.
  std::map<std::string, const ValueInfo*> gin;
  for (auto& vi : g.inputs) gin[vi.name] = &vi;
  size_t total = 0;
  for (auto& t : g.inits) total += (t.f32.size() * 4 + 255) / 256 * 256;
  std::vector<char> host(total ? total : 1, 0);
  if (total && hipMalloc(reinterpret_cast<void**>(&m->consts), total) != hipSuccess)
    return fail(set_error(ctx, ORE_ERR_OOM, "initializer upload allocation failed"));
  size_t off = 0;
  for (auto& t : g.inits) {
    int id = new_value(m, t.name);
    Value& v = m->values[id];
    v.is_const = true;
    std::vector<int64_t> shape = t.dims;
    auto it = gin.find(t.name);
    if (it != gin.end() && !it->second->shape.empty()) shape = it->second->shape;
    if (shape.size() > 4) return fail(set_error(ctx, ORE_ERR_UNSUPPORTED, "initializer '%s' rank > 4", t.name.c_str()));
    v.ndim = int(shape.size());
    for (size_t i = 0; i < shape.size(); ++i) v.dims[i] = shape[i];
    if (!t.f32.empty()) {
      if (int64_t(t.f32.size()) != v.numel_const())
        return fail(set_error(ctx, ORE_ERR_INVALID, "initializer '%s' has %zu values for its shape", t.name.c_str(), t.f32.size()));
      std::memcpy(host.data() + off, t.f32.data(), t.f32.size() * 4);
      v.cptr = reinterpret_cast<float*>(reinterpret_cast<char*>(m->consts) + off);
      off += (t.f32.size() * 4 + 255) / 256 * 256;
    }
    if (!t.i64.empty()) { v.i64 = t.i64; v.has_i64 = true; }
  }
  if (total) {
    if (hipMemcpy(m->consts, host.data(), total, hipMemcpyHostToDevice) != hipSuccess)
      return fail(set_error(ctx, ORE_ERR_HIP, "initializer upload failed"));
  }
  // seeded input (manage_input_data, utils.rs:29-45): graph inputs that are not initializers
  for (auto& vi : g.inputs) {
    if (value_id(m, vi.name) >= 0) continue;
    if (m->input_value >= 0) return fail(set_error(ctx, ORE_ERR_UNSUPPORTED, "more than one seeded model input"));
    if (vi.shape.size() != 4) return fail(set_error(ctx, ORE_ERR_UNSUPPORTED, "model input '%s' must be 4-D", vi.name.c_str()));
    int id = new_value(m, vi.name);
    Value& v = m->values[id];
    v.is_input = true;
    v.ndim = 4;
    v.dims[0] = 1;
    for (int i = 1; i < 4; ++i) {
      if (vi.shape[i] <= 0) return fail(set_error(ctx, ORE_ERR_UNSUPPORTED, "symbolic input dims are not supported"));
      v.dims[i] = vi.shape[i];
    }
    m->input_value = id;
  }
  if (m->input_value < 0) return fail(set_error(ctx, ORE_ERR_UNSUPPORTED, "model has no seeded input"));
  for (auto& n : g.nodes) {
    Step s;
    ore_status st = build_node(m, n, &s);
    if (st) { std::string e = ctx->err; ore_model_destroy(m); return set_error(ctx, st, "%s", e.c_str()); }
    m->base_steps.push_back(s);
  }
  // pack every conv / matmul weight once (K-major, zero padded) for the MFMA A tiles
  {
    size_t total_packed = 0;
    for (auto& s : m->base_steps) {
      if (s.kind == S_CONV) {
        // f16 operand mode by the input's layout: an f32 NCHW value (the model input: converted to
        // NHWC4 when C <= 4, else gathered per element), or NHWC f16 (16-B channel groups when C % 8 == 0)
        // (SqueezeNet conv1 at B = 256: NHWC4 pairs 355 us, per-element NCHW 459 us,
        // profiles/r01p_f16_first_conv.txt)
        const int xmode = m->values[s.in0].es == 4 ? (s.C <= 4 ? F16_X_NHWC_PAIR : F16_X_NCHW32)
                          : s.C % 8 == 0           ? F16_X_NHWC_VEC
                                                   : F16_X_NHWC_ELEM;
        s.plan = conv_plan(s.M, s.C, s.H, s.W, s.kh, s.kw, s.sh, s.sw, s.win, m->f16, xmode, false, m->conv_tile);
      }
      else if (s.kind == S_MATMUL)
        s.plan = conv_plan(s.M, s.C, 1, 1, 1, 1, 1, 1, s.win, false, 0, false, m->conv_tile);
      else
        continue;
      total_packed += (packed_bytes(s.plan) + 255) / 256 * 256;
      if (m->wino && s.kind == S_CONV) {
        s.plan_wino = conv_plan(s.M, s.C, s.H, s.W, s.kh, s.kw, s.sh, s.sw, s.win, false, 0, true, m->conv_tile);
        s.has_wino = s.plan_wino.wino != 0;
        if (s.has_wino) total_packed += (conv_packed_bytes(s.plan_wino) + 255) / 256 * 256;
      }
    }
    if (total_packed) {
      if (hipMalloc(reinterpret_cast<void**>(&m->packed), total_packed) != hipSuccess)
        return fail(set_error(ctx, ORE_ERR_OOM, "packed weight allocation failed"));
      size_t poff = 0;
      for (auto& s : m->base_steps) {
        if (s.kind != S_CONV && s.kind != S_MATMUL) continue;
        char* base = reinterpret_cast<char*>(m->packed) + poff;
        s.wp = reinterpret_cast<float*>(base);
        launch_pack(m->values[s.in1].cptr, s.w_kmajor, int(s.M), int(s.C), int(s.kh), int(s.kw), s.plan, s.wp,
                    ctx->stream);
        s.ktab = reinterpret_cast<int2*>(base + conv_packed_bytes(s.plan));
        poff += (packed_bytes(s.plan) + 255) / 256 * 256;
        if (s.has_wino) {
          s.wp_wino = reinterpret_cast<float*>(reinterpret_cast<char*>(m->packed) + poff);
          launch_pack(m->values[s.in1].cptr, false, int(s.M), int(s.C), int(s.kh), int(s.kw), s.plan_wino, s.wp_wino,
                      ctx->stream);
          poff += (conv_packed_bytes(s.plan_wino) + 255) / 256 * 256;
        }
      }
      if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess)
        return fail(set_error(ctx, ORE_ERR_HIP, "weight packing failed"));
    }
  }
  if (g.outputs.empty()) return fail(set_error(ctx, ORE_ERR_INVALID, "model has no outputs"));
  m->output_value = value_id(m, g.outputs[0].name);
  if (m->output_value < 0 || m->values[m->output_value].is_const)
    return fail(set_error(ctx, ORE_ERR_INVALID, "graph output '%s' is not produced", g.outputs[0].name.c_str()));
  m->values[m->output_value].is_output = true;
  if (m->values[m->output_value].es != 4)
    return fail(set_error(ctx, ORE_ERR_UNSUPPORTED, "f16 model: graph output '%s' must be f32 (end with GlobalAveragePool / Softmax)",
                          g.outputs[0].name.c_str()));
  if (ore_status st = plan(m)) { std::string e = ctx->err; ore_model_destroy(m); return set_error(ctx, st, "%s", e.c_str()); }
  *out = m;
  return ORE_OK;
}

ore_status ore_model_destroy(ore_model* m) {
  if (!m) return ORE_OK;
  (void)hipSetDevice(m->ctx->device);
  (void)hipStreamSynchronize(m->ctx->stream);
  for (auto e : m->events) (void)hipEventDestroy(e);
  if (m->graph_exec) (void)hipGraphExecDestroy(m->graph_exec);
  if (m->graph) (void)hipGraphDestroy(m->graph);
  if (m->side) (void)hipStreamDestroy(m->side);
  if (m->ev_fork) (void)hipEventDestroy(m->ev_fork);
  if (m->ev_join) (void)hipEventDestroy(m->ev_join);
  if (m->arena_alloc) (void)hipFree(m->arena_alloc);
  if (m->consts) (void)hipFree(m->consts);
  if (m->packed) (void)hipFree(m->packed);
  for (auto& kv : m->fire_packs) (void)hipFree(kv.second);
  if (m->xcvt) (void)hipFree(m->xcvt);
  delete m;
  return ORE_OK;
}

ore_status ore_model_set_fusion(ore_model* m, int32_t flags) {
  if (!m) return set_error(nullptr, ORE_ERR_INVALID, "null model");
  const int32_t known = ORE_FUSE_ALL | ORE_FUSE_EAGER | ORE_KEEP_VALUES;
  if (flags & 16) return set_error(m->ctx, ORE_ERR_UNSUPPORTED, "fusion bit 16 (ORE_FUSE_POOL_CONV) was retired (ABI 2)");
  if (flags & ~known) return set_error(m->ctx, ORE_ERR_INVALID, "unknown fusion flags 0x%x", unsigned(flags & ~known));
  m->fusion = flags;
  return plan(m);
}

ore_status ore_model_input_dims(ore_model* m, int64_t dims[4]) {
  if (!m || !dims) return set_error(nullptr, ORE_ERR_INVALID, "null argument");
  for (int i = 0; i < 4; ++i) dims[i] = m->values[m->input_value].dims[i];
  return ORE_OK;
}

ore_status ore_model_output_elems(ore_model* m, int64_t* elems) {
  if (!m || !elems) return set_error(nullptr, ORE_ERR_INVALID, "null argument");
  *elems = m->values[m->output_value].per_image();
  return ORE_OK;
}

// one pass of the graph over n <= run_batch images; ev: this pass's timing events (exec_steps + 1)
static ore_status run_pass(ore_model* m, const float* d_input, int64_t n, float* d_output, hipEvent_t* ev) {
  ore_ctx* ctx = m->ctx;
  m->cur_in = d_input;
  m->cur_out = d_output;
  const Value& ov = m->values[m->output_value];
  const bool branches = m->streams > 1 && !m->timing;
  for (size_t k = 0; k < m->exec_steps.size(); ++k) {
    if (m->timing) ORE_HIP_CHECK(ctx, hipEventRecord(ev[k], ctx->stream));
    if (branches && m->pair_next[k]) {
      // fork: step k on the side stream, step k + 1 on the main stream, then join
      ORE_HIP_CHECK(ctx, hipEventRecord(m->ev_fork, ctx->stream));
      ORE_HIP_CHECK(ctx, hipStreamWaitEvent(m->side, m->ev_fork, 0));
      hipStream_t main = ctx->stream;
      ctx->stream = m->side;
      ore_status st = launch_step(m, m->steps[m->exec_steps[k]], n);
      ctx->stream = main;
      if (st) return st;
      ORE_HIP_CHECK(ctx, hipEventRecord(m->ev_join, m->side));
      st = launch_step(m, m->steps[m->exec_steps[k + 1]], n);
      if (st) return st;
      ORE_HIP_CHECK(ctx, hipStreamWaitEvent(ctx->stream, m->ev_join, 0));
      ++k;
      continue;
    }
    ore_status st = launch_step(m, m->steps[m->exec_steps[k]], n);
    if (st) return st;
  }
  if (m->timing) ORE_HIP_CHECK(ctx, hipEventRecord(ev[m->exec_steps.size()], ctx->stream));
  if (!m->out_bound) {
    const Ref r = ref_of(m, m->output_value);
    const int64_t pe = ov.per_image();
    if (r.nstride == pe) {
      ORE_HIP_CHECK(ctx, hipMemcpyAsync(d_output, r.p, size_t(n * pe) * 4, hipMemcpyDeviceToDevice, ctx->stream));
    } else {
      ORE_HIP_CHECK(ctx, hipMemcpy2DAsync(d_output, size_t(pe) * 4, r.p, size_t(r.nstride) * 4, size_t(pe) * 4, size_t(n),
                                          hipMemcpyDeviceToDevice, ctx->stream));
    }
  }
  return ORE_OK;
}

ore_status ore_model_run(ore_model* m, const float* d_input, int64_t n, float* d_output) {
  if (!m || !d_input || !d_output) return set_error(m ? m->ctx : nullptr, ORE_ERR_INVALID, "null argument");
  ore_ctx* ctx = m->ctx;
  if (n < 0 || n > m->max_batch) return set_error(ctx, ORE_ERR_INVALID, "batch %lld exceeds max_batch %lld", (long long)n, (long long)m->max_batch);
  ORE_HIP_CHECK(ctx, hipSetDevice(ctx->device));
  m->last_n = n;
  const Value& ov = m->values[m->output_value];
  // bind the output buffer directly when its producer writes a plain contiguous tensor
  m->out_bound = ov.alias_of < 0 && !ov.elided;
  // n > run_batch: equal chunks of consecutive images, at most run_batch each (every image's
  // arithmetic is independent of the batch it runs in)
  const int64_t nchunks = n > m->run_batch ? (n + m->run_batch - 1) / m->run_batch : 1;
  const int64_t chunk = (n + nchunks - 1) / nchunks;
  m->last_chunked = nchunks > 1;
  const size_t nev = m->exec_steps.size() + 1;
  if (m->timing && m->events.size() < nev * size_t(nchunks)) {
    for (auto e : m->events) (void)hipEventDestroy(e);
    m->events.assign(nev * size_t(nchunks), nullptr);
    for (auto& e : m->events) ORE_HIP_CHECK(ctx, hipEventCreate(&e));
  }
  m->timed_chunks = m->timing ? int(nchunks) : 0;
  if (m->streams > 1 && !m->timing && !m->side) {
    ORE_HIP_CHECK(ctx, hipStreamCreateWithFlags(&m->side, hipStreamNonBlocking));
    ORE_HIP_CHECK(ctx, hipEventCreateWithFlags(&m->ev_fork, hipEventDisableTiming));
    ORE_HIP_CHECK(ctx, hipEventCreateWithFlags(&m->ev_join, hipEventDisableTiming));
  }
  const int64_t in_img = m->values[m->input_value].per_image(), out_img = ov.per_image();
  for (int64_t c = 0, i0 = 0; c < nchunks; ++c, i0 += chunk) {
    const int64_t nc = std::min(chunk, n - i0);
    if (ore_status st = run_pass(m, d_input + i0 * in_img, nc, d_output + i0 * out_img,
                                 m->timing ? m->events.data() + size_t(c) * nev : nullptr))
      return st;
  }
  return ORE_OK;
}

ore_status ore_model_read_value(ore_model* m, const char* name, float* host_dst, size_t cap, int64_t dims[4],
                                int32_t* ndim) {
  if (!m || !name) return set_error(nullptr, ORE_ERR_INVALID, "null argument");
  ore_ctx* ctx = m->ctx;
  int id = value_id(m, name);
  if (id < 0) return set_error(ctx, ORE_ERR_INVALID, "no value named '%s'", name);
  const Value& v = m->values[id];
  if (v.elided) return set_error(ctx, ORE_ERR_INVALID, "value '%s' is fused away", name);
  if (!v.is_const && m->last_chunked)
    return set_error(ctx, ORE_ERR_INVALID, "the last run went in image chunks of %lld: value '%s' holds only the last one",
                     (long long)m->run_batch, name);
  const int64_t n = v.is_const ? 1 : m->last_n;
  if (dims) {
    for (int i = 0; i < 4; ++i) dims[i] = v.dims[i];
    if (!v.is_const) dims[0] = n;
  }
  if (ndim) *ndim = v.ndim;
  const int64_t pe = v.is_const ? v.numel_const() : v.per_image();
  if (!host_dst) return ORE_OK;
  if (size_t(n * pe) > cap) return set_error(ctx, ORE_ERR_INVALID, "destination too small");
  {
    int rid = id;
    while (m->values[rid].alias_of >= 0) rid = m->values[rid].alias_of;
    const Value& rv = m->values[rid];
    if (!rv.is_const && rv.first < 0 && !rv.is_input)
      return set_error(ctx, ORE_ERR_INVALID, "value '%s' not materialised", name);
    // Without ORE_KEEP_VALUES the arena reuses slots by liveness: a value whose bytes a later value
    // (first write after this one's last read) overlaps was overwritten during the run -> refuse
    // rather than return stale data.
    if (!(m->fusion & ORE_KEEP_VALUES) && rv.arena_off >= 0) {
      auto extent = [&](const Value& x) {
        return ((x.image_stride() * m->run_batch * x.es) + 255) / 256 * 256;
      };
      const int64_t lo = rv.arena_off, hi = rv.arena_off + extent(rv);
      for (size_t j = 0; j < m->values.size(); ++j) {
        const Value& o = m->values[j];
        if (int(j) == rid || o.arena_off < 0 || o.alias_of >= 0 || o.is_const || o.is_input || o.elided) continue;
        if (o.first > rv.last && o.arena_off < hi && lo < o.arena_off + extent(o))
          return set_error(ctx, ORE_ERR_INVALID,
                           "value '%s' was overwritten by a later value in the arena (load with ORE_KEEP_VALUES "
                           "to read intermediate values)", name);
      }
    }
  }
  ORE_HIP_CHECK(ctx, hipSetDevice(ctx->device));
  ORE_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
  const Ref r = ref_of(m, id);
  if (!r.p) return set_error(ctx, ORE_ERR_INVALID, "value '%s' has no f32 storage", name);
  const int64_t ns = v.is_const ? pe : r.nstride;
  if (r.es == 2) {  // f16 storage: download the halves, convert (and, channels-last, transpose) on the host
    std::vector<uint16_t> tmp(size_t(n * pe));
    if (v.nhwc) {  // per image: H*W pixels of C channels at pixel stride ps -> NCHW
      const int64_t C = v.dims[1], HW = v.dims[2] * v.dims[3];
      for (int64_t i = 0; i < n; ++i)
        ORE_HIP_CHECK(ctx, hipMemcpy2D(tmp.data() + i * pe, size_t(C) * 2, reinterpret_cast<const char*>(r.p) + i * ns * 2,
                                       size_t(r.ps) * 2, size_t(C) * 2, size_t(HW), hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < n; ++i)
        for (int64_t q = 0; q < HW; ++q)
          for (int64_t c = 0; c < C; ++c) host_dst[i * pe + c * HW + q] = half_bits_to_float(tmp[size_t(i * pe + q * C + c)]);
      return ORE_OK;
    }
    ORE_HIP_CHECK(ctx, hipMemcpy2D(tmp.data(), size_t(pe) * 2, r.p, size_t(ns) * 2, size_t(pe) * 2, size_t(n),
                                   hipMemcpyDeviceToHost));
    for (size_t i = 0; i < tmp.size(); ++i) host_dst[i] = half_bits_to_float(tmp[i]);
    return ORE_OK;
  }
  if (!v.is_const && v.ndim == 4 && r.ps && r.ps != v.dims[2] * v.dims[3]) {  // padded planes
    const int64_t P = v.dims[2] * v.dims[3];
    for (int64_t i = 0; i < n; ++i)
      ORE_HIP_CHECK(ctx, hipMemcpy2D(host_dst + i * pe, size_t(P) * 4, r.p + i * ns, size_t(r.ps) * 4, size_t(P) * 4,
                                     size_t(v.dims[1]), hipMemcpyDeviceToHost));
    return ORE_OK;
  }
  ORE_HIP_CHECK(ctx, hipMemcpy2D(host_dst, size_t(pe) * 4, r.p, size_t(ns) * 4, size_t(pe) * 4, size_t(n),
                                 hipMemcpyDeviceToHost));
  return ORE_OK;
}

ore_status ore_model_autotune(ore_model* m, const float* d_input, int64_t n, float* d_output, int32_t reps) {
  if (!m || !d_input || !d_output) return set_error(m ? m->ctx : nullptr, ORE_ERR_INVALID, "null argument");
  ore_ctx* ctx = m->ctx;
  if (n < 1 || n > m->max_batch) return set_error(ctx, ORE_ERR_INVALID, "batch out of range");
  if (reps < 1) reps = 3;
  const int64_t n_all = n;
  if (n > m->run_batch) {  // tuned on one chunk of the chunked run (ore_model_run)
    const int64_t nchunks = (n + m->run_batch - 1) / m->run_batch;
    n = (n + nchunks - 1) / nchunks;
  }
  m->last_chunked = false;
  ORE_HIP_CHECK(ctx, hipSetDevice(ctx->device));
  m->cur_in = d_input;
  m->cur_out = d_output;
  m->last_n = n;
  const Value& ov = m->values[m->output_value];
  m->out_bound = ov.alias_of < 0 && !ov.elided;
  hipEvent_t e0, e1;
  ORE_HIP_CHECK(ctx, hipEventCreate(&e0));
  ORE_HIP_CHECK(ctx, hipEventCreate(&e1));
  ore_status st = ORE_OK;
  // steps run in order so every conv sees its real input geometry; each candidate tile is timed on
  // the step's own buffers and the fastest kept (results do not depend on the tile: every output is
  // the same k-ordered MFMA chain, every pooled value the same max)
  for (size_t k = 0; k < m->exec_steps.size() && !st; ++k) {
    Step& s = m->steps[m->exec_steps[k]];
    const std::vector<int> cands = step_tile_family(s);
    if (cands.size() < 2) {
      if (cands.size() == 1) set_tile(m, int(k), cands[0]);
      st = launch_step(m, s, n);
      continue;
    }
    int best = -1;
    float best_ms = 1e30f;
    for (size_t ci = 0; ci < cands.size() && !st; ++ci) {
      const int c = cands[ci];
      set_tile(m, int(k), c);
      last_conv_tile = -1;
      st = launch_step(m, s, n);  // warm-up
      if (st) break;
      if (last_conv_tile != c) continue;  // fell back to another kernel: not a distinct candidate here
      if (hipEventRecord(e0, ctx->stream) != hipSuccess) { st = set_error(ctx, ORE_ERR_HIP, "event record"); break; }
      for (int r = 0; r < reps && !st; ++r) st = launch_step(m, s, n);
      if (st) break;
      float ms = 0.f;
      if (hipEventRecord(e1, ctx->stream) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
          hipEventElapsedTime(&ms, e0, e1) != hipSuccess) {
        st = set_error(ctx, ORE_ERR_HIP, "autotune timing failed");
        break;
      }
      if (ms < best_ms) { best_ms = ms; best = c; }
    }
    if (best >= 0) set_tile(m, int(k), best);
    if (!st) st = launch_step(m, s, n);  // leave the real output for the next step
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (!st && hipStreamSynchronize(ctx->stream) != hipSuccess) st = set_error(ctx, ORE_ERR_HIP, "autotune sync");
  // tuned on the first chunk only: run the whole batch once so d_output holds every image's output
  if (!st && n_all > n) st = ore_model_run(m, d_input, n_all, d_output);
  if (!st && n_all > n && hipStreamSynchronize(ctx->stream) != hipSuccess) st = set_error(ctx, ORE_ERR_HIP, "autotune sync");
  return st;
}

int32_t ore_model_step_tile(ore_model* m, int32_t i) {
  if (!m || i < 0 || size_t(i) >= m->exec_steps.size()) return -1;
  const Step& s = m->steps[m->exec_steps[i]];
  if (s.kind == S_FIRE) return s.fire_f16 ? FIRE_F16_TILE : s.fire_pool ? FIRE_POOL_TILE : FIRE_TILE;
  if (s.kind == S_CONV && s.epool && !s.plan.f16 && s.plan.epv > 0) return epool_tile_id(s.plan.epv);
  if (s.kind == S_CONV && s.epool && s.ran_tile >= 0) return s.ran_tile;
  if (s.kind == S_CONV && s.gap) return s.plan.f16 ? CONV_GAP_F16_TILE : CONV_GAP_F32_TILE;
  return (s.kind == S_CONV || s.kind == S_MATMUL) ? s.plan.cfg : -1;
}

ore_status ore_model_set_step_tile(ore_model* m, int32_t i, int32_t tile) {
  if (!m || i < 0 || size_t(i) >= m->exec_steps.size()) return set_error(m ? m->ctx : nullptr, ORE_ERR_INVALID, "bad step index");
  const std::vector<int> fam = step_tile_family(m->steps[m->exec_steps[i]]);
  if (std::find(fam.begin(), fam.end(), int(tile)) == fam.end())
    return set_error(m->ctx, ORE_ERR_INVALID, "tile %d is not a kernel of step %d ('%s')", int(tile), int(i),
                     m->steps[m->exec_steps[i]].name.c_str());
  set_tile(m, i, tile);
  return ORE_OK;
}

ore_status ore_model_step_mfma_flops(ore_model* m, int32_t i, double* flops) {
  if (!m || !flops || i < 0 || size_t(i) >= m->exec_steps.size())
    return set_error(m ? m->ctx : nullptr, ORE_ERR_INVALID, "bad step index");
  const Step& s = m->steps[m->exec_steps[i]];
  *flops = (s.mfma_flops_per_img >= 0 ? s.mfma_flops_per_img : s.flops_per_img) * double(m->last_n);
  return ORE_OK;
}

ore_status ore_model_set_streams(ore_model* m, int32_t streams) {
  if (!m || streams < 1 || streams > 2) return set_error(m ? m->ctx : nullptr, ORE_ERR_INVALID, "streams must be 1 or 2");
  m->streams = streams;
  return ORE_OK;
}

ore_status ore_model_graph_capture(ore_model* m, const float* d_input, int64_t n, float* d_output) {
  if (!m || !d_input || !d_output) return set_error(m ? m->ctx : nullptr, ORE_ERR_INVALID, "null argument");
  ore_ctx* ctx = m->ctx;
  if (m->timing) return set_error(ctx, ORE_ERR_INVALID, "disable step timing before capturing a graph");
  if (!ctx->stream) return set_error(ctx, ORE_ERR_INVALID, "graph capture needs a non-null context stream");
  ORE_HIP_CHECK(ctx, hipSetDevice(ctx->device));
  if (m->graph_exec) { (void)hipGraphExecDestroy(m->graph_exec); m->graph_exec = nullptr; }
  if (m->graph) { (void)hipGraphDestroy(m->graph); m->graph = nullptr; }
  if (m->streams > 1 && !m->side) {  // created outside the capture
    ORE_HIP_CHECK(ctx, hipStreamCreateWithFlags(&m->side, hipStreamNonBlocking));
    ORE_HIP_CHECK(ctx, hipEventCreateWithFlags(&m->ev_fork, hipEventDisableTiming));
    ORE_HIP_CHECK(ctx, hipEventCreateWithFlags(&m->ev_join, hipEventDisableTiming));
  }
  ORE_HIP_CHECK(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
  ore_status st = ore_model_run(m, d_input, n, d_output);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(ctx->stream, &g);
  if (st) {
    if (g) (void)hipGraphDestroy(g);
    return st;
  }
  if (e != hipSuccess) return set_error(ctx, ORE_ERR_HIP, "hipStreamEndCapture: %s", hipGetErrorString(e));
  m->graph = g;
  ORE_HIP_CHECK(ctx, hipGraphInstantiate(&m->graph_exec, m->graph, nullptr, nullptr, 0));
  return ORE_OK;
}

ore_status ore_model_graph_launch(ore_model* m) {
  if (!m) return set_error(nullptr, ORE_ERR_INVALID, "null model");
  if (!m->graph_exec) return set_error(m->ctx, ORE_ERR_INVALID, "no captured graph (ore_model_graph_capture)");
  ORE_HIP_CHECK(m->ctx, hipGraphLaunch(m->graph_exec, m->ctx->stream));
  return ORE_OK;
}

ore_status ore_model_enable_timing(ore_model* m, int32_t on) {
  if (!m) return set_error(nullptr, ORE_ERR_INVALID, "null model");
  m->timing = on != 0;
  return ORE_OK;
}

int32_t ore_model_step_count(ore_model* m) { return m ? int32_t(m->exec_steps.size()) : 0; }

int64_t ore_model_run_batch(ore_model* m) { return m ? m->run_batch : 0; }

ore_status ore_model_step_info(ore_model* m, int32_t i, const char** op, const char** name, double* flops, double* bytes) {
  if (!m || i < 0 || size_t(i) >= m->exec_steps.size()) return set_error(nullptr, ORE_ERR_INVALID, "bad step index");
  const Step& s = m->steps[m->exec_steps[i]];
  static const char* kinds[] = {"Conv", "MaxPool", "Relu", "Add", "Softmax", "MatMul", "GlobalAveragePool", "Concat", "Copy",
                                "Nop", "Conv"};  // S_FIRE: three convs (expand 1x1 / 3x3 + squeeze) in one launch
  if (op) *op = kinds[s.kind];
  if (name) *name = s.name.c_str();
  const double n = double(m->last_n);
  if (flops) *flops = s.flops_per_img * n;
  if (bytes) {
    double b = s.bytes_per_img * n + s.bytes_fixed;
    // fused epilogues/in-place writes move fewer bytes than the op-by-op accounting
    *bytes = b;
  }
  return ORE_OK;
}

ore_status ore_model_step_times(ore_model* m, float* ms, int32_t cap) {
  if (!m || !ms) return set_error(nullptr, ORE_ERR_INVALID, "null argument");
  const size_t nev = m->exec_steps.size() + 1;
  if (!m->timing || m->timed_chunks < 1 || m->events.size() < nev * size_t(m->timed_chunks))
    return set_error(m->ctx, ORE_ERR_INVALID, "timing not enabled");
  ORE_HIP_CHECK(m->ctx, hipEventSynchronize(m->events[nev * size_t(m->timed_chunks) - 1]));
  for (size_t k = 0; k < m->exec_steps.size() && int32_t(k) < cap; ++k) {
    ms[k] = 0.f;
    for (int c = 0; c < m->timed_chunks; ++c) {  // summed over the run's image chunks
      float t = 0.f;
      ORE_HIP_CHECK(m->ctx, hipEventElapsedTime(&t, m->events[c * nev + k], m->events[c * nev + k + 1]));
      ms[k] += t;
    }
  }
  return ORE_OK;
}

}  // extern "C"
