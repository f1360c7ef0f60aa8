// gfx950 kernels of the ENet range coder: the `Compressor`
// implementation `RangeCoder` of jabuwu/rusty_enet (src/compressor.rs:36-69) over
// src/c/compress.rs, batched across packets.
//
// The coder is sequential inside a packet (every symbol updates the adaptive
// order-2 model that codes the next one), so the parallelism is across packets:
// one lane = one coder = one packet at a time (grid-stride over the batch).
// Each lane owns a 64 KiB symbol arena (4096 x 16-B ENetSymbol, compress.rs:7-22)
// in HBM scratch.  A symbol is read as ONE 16-byte load; updates store whole
// 32-bit words rebuilt from the loaded copy.  The work is a chain of dependent arena
// loads (tree walks in up to three contexts per byte), so the kernel is
// latency-bound, not bandwidth-bound: throughput comes from the number of lanes
// in flight (the `workers` argument sizes the scratch and the grid).
//
// Semantics follow compress.rs statement for statement (line numbers below),
// including the u16/u8 wrap-around of every counter and the arena reset at
// 4094 symbols (:426-450).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "range_coder.hpp"

namespace enet_crc {
namespace {

constexpr uint32_t kSymbolMinimum = 1;   // compress.rs:23
constexpr uint32_t kEscapeMinimum = 1;   // :24
constexpr uint32_t kOrder = 2;           // :25
constexpr uint32_t kBottom = 65536;      // :26
constexpr uint32_t kSubSymbolDelta = 2;  // :27
constexpr uint32_t kSubEscapeDelta = 5;  // :28
constexpr uint32_t kCtxSymbolDelta = 3;  // :29
constexpr uint32_t kTop = 16777216;      // :30
constexpr uint32_t kArena = 4096;        // :8
constexpr int kBlock = 256;

// Debug hooks: RC_DECODE_ATTR / RC_MODEL_ATTR (e.g. optnone / noinline) for A/B builds.
// History: an earlier version with byte/short stores into an ENetSymbol struct decoded
// wrong symbols on gfx950 at -O1 and above (bit-exact at -O0 and on the host); the
// whole-word layout below is bit-exact optimised (tools/dbg/standalone.hip).
#ifndef RC_DECODE_ATTR
#define RC_DECODE_ATTR
#endif
#ifndef RC_MODEL_ATTR
#define RC_MODEL_ATTR
#endif

// Decoder exit codes (debug builds only: -DRC_DEBUG_EXITS makes the decoder report
// which exit it took instead of the reference's 0).
#ifdef RC_DEBUG_EXITS
#define RC_FAIL(reason, n) (0x7F000000u | ((reason) << 16) | ((n) & 0xFFFF))
#else
#define RC_FAIL(reason, n) 0u
#endif

// ENetSymbol (compress.rs:12-22) as four 32-bit words, the same 16 bytes:
//   x = value | count << 8 | under << 16     y = left | right << 16
//   z = symbols | escapes << 16              w = total | parent << 16
// A node is read with one 16-byte load; every update stores whole words rebuilt from
// the loaded copy (no byte/short stores).
using Sym = uint4;
static_assert(sizeof(Sym) == 16, "ENetSymbol is 16 bytes");
static_assert(kArena * sizeof(Sym) == kRangeArenaBytes, "arena size");

__host__ __device__ inline uint32_t lo16(uint32_t v) { return v & 0xFFFF; }
__host__ __device__ inline uint32_t hi16(uint32_t v) { return v >> 16; }
__host__ __device__ inline uint32_t pack(uint32_t lo, uint32_t hi) { return (lo & 0xFFFF) | (hi << 16); }
__host__ __device__ inline uint32_t sym_value(const Sym& s) { return s.x & 0xFF; }
__host__ __device__ inline uint32_t sym_count(const Sym& s) { return (s.x >> 8) & 0xFF; }
__host__ __device__ inline uint32_t sym_x(uint32_t value, uint32_t count, uint32_t under) {
  return (value & 0xFF) | ((count & 0xFF) << 8) | (under << 16);
}

struct Model {
  Sym* a;
  uint32_t next;
  uint32_t predicted;
  uint32_t order;

  __host__ __device__ Sym load(uint32_t i) const { return a[i]; }
  __host__ __device__ uint32_t* words(uint32_t i) const { return reinterpret_cast<uint32_t*>(a + i); }

  RC_MODEL_ATTR __host__ __device__ uint32_t new_symbol(uint32_t value, uint32_t delta) {
    const uint32_t i = next++;
    a[i] = Sym{sym_x(value, delta, delta), 0u, 0u, 0u};
    return i;
  }

  // compress.rs:86-101 / :426-450
  RC_MODEL_ATTR __host__ __device__ void reset() {
    a[0] = Sym{0u, 0u, pack(0, kEscapeMinimum), pack(kEscapeMinimum + 256 * kSymbolMinimum, 0)};
    next = 1;
    predicted = 0;
    order = 0;
  }

  // `parent` chain target: ~0u = the `predicted` register, else the .parent field of a symbol.
  RC_MODEL_ATTR __host__ __device__ void set_parent(uint32_t slot, uint32_t v) {
    if (slot == ~0u) {
      predicted = v;
    } else {
      uint32_t* w = words(slot);
      w[3] = pack(w[3], v);
    }
  }

  // enet_symbol_rescale, compress.rs:42-59, with the left recursion on an explicit
  // stack (a context tree has at most 256 nodes).  Stack entry = node | frame total << 16.
  RC_MODEL_ATTR __host__ __device__ uint32_t rescale(uint32_t i) {
    uint32_t stk[256];
    int sp = 0;
    uint32_t total = 0;
    for (;;) {
      Sym s = load(i);
      const uint32_t c0 = sym_count(s);
      const uint32_t c = c0 - (c0 >> 1);
      s.x = sym_x(sym_value(s), c, c);
      words(i)[0] = s.x;
      if (lo16(s.y)) {  // descend; finish this node after the left subtree returns
        stk[sp++] = i | (total << 16);
        i += lo16(s.y);
        total = 0;
        continue;
      }
      total = (total + c) & 0xFFFF;
      // walk right; when a frame ends, return its total to the node that pushed it
      for (;;) {
        if (hi16(s.y)) {
          i += hi16(s.y);
          break;
        }
        if (sp == 0) return total;
        const uint32_t e = stk[--sp];
        const uint32_t sub = total;
        i = e & 0xFFFF;
        total = e >> 16;
        s = load(i);
        const uint32_t u = (hi16(s.x) + sub) & 0xFFFF;
        s.x = pack(s.x, u);
        words(i)[0] = s.x;
        total = (total + u) & 0xFFFF;
      }
    }
  }

  // find-or-insert `value` in context ctx's tree (compress.rs:137-212, :301-376, :847-922).
  RC_MODEL_ATTR __host__ __device__ uint32_t update(uint32_t ctx, uint32_t value, uint32_t delta, uint32_t& under,
                                                    uint32_t& count) {
    const uint32_t cz = words(ctx)[2];
    if (lo16(cz) == 0) {
      const uint32_t n = new_symbol(value, delta);
      words(ctx)[2] = pack(n - ctx, hi16(cz));
      return n;
    }
    uint32_t i = ctx + lo16(cz);
    for (;;) {
      const Sym s = load(i);
      const uint32_t v = sym_value(s);
      if (value < v) {
        words(i)[0] = pack(s.x, hi16(s.x) + delta);
        if (lo16(s.y)) {
          i += lo16(s.y);
          continue;
        }
        const uint32_t n = new_symbol(value, delta);
        words(i)[1] = pack(n - i, hi16(s.y));
        return n;
      }
      if (value > v) {
        under = (under + hi16(s.x)) & 0xFFFF;
        if (hi16(s.y)) {
          i += hi16(s.y);
          continue;
        }
        const uint32_t n = new_symbol(value, delta);
        words(i)[1] = pack(s.y, n - i);
        return n;
      }
      const uint32_t c = sym_count(s), u = hi16(s.x);
      count = (count + c) & 0xFFFF;
      under = (under + u - c) & 0xFFFF;
      words(i)[0] = sym_x(v, c + delta, (u + delta) & 0xFFFF);
      return i;
    }
  }

  // context rescale, :276-289 (root: :404-419, extra = 256 * SYMBOL_MINIMUM)
  RC_MODEL_ATTR __host__ __device__ void ctx_rescale(uint32_t ctx, uint32_t extra) {
    const Sym c = load(ctx);
    const uint32_t t = lo16(c.z) ? rescale(ctx + lo16(c.z)) : 0;
    const uint32_t e = hi16(c.z) - (hi16(c.z) >> 1);
    words(ctx)[2] = pack(c.z, e);
    words(ctx)[3] = pack(t + e + extra, hi16(c.w));
  }

  // :421-450, after every symbol
  RC_MODEL_ATTR __host__ __device__ void advance() {
    if (order >= kOrder)
      predicted = hi16(words(predicted)[3]);
    else
      ++order;
    if (next >= kArena - kOrder) reset();
  }
};

struct Encoder {
  uint32_t low = 0, range = ~0u;
  uint8_t* out;
  uint8_t* end;
  // encode + renormalise, e.g. compress.rs:217-241; false = output limit reached
  __host__ __device__ bool put(uint32_t under, uint32_t count, uint32_t total) {
    range /= total;
    low += under * range;
    range *= count;
    for (;;) {
      if ((low ^ (low + range)) >= kTop) {
        if (range >= kBottom) return true;
        range = (0u - low) & (kBottom - 1);
      }
      if (out >= end) return false;
      *out++ = (uint8_t)(low >> 24);
      range <<= 8;
      low <<= 8;
    }
  }
};

// enet_range_coder_compress over one contiguous input (compress.rs:60-462), as a
// resumable per-lane state machine: begin() sets a packet up, step() codes ONE input
// byte and reports whether the packet is finished (its result in `size`).  The kernel
// calls step() in a loop and starts the lane's next packet as soon as one finishes,
// so a lane never idles while the longest packet of its wave is still being coded.
struct CompressLane {
  const uint8_t* in;
  uint32_t pos, len, size;
  uint8_t* out0;
  Encoder e;

  __host__ __device__ void begin(Model& m, const uint8_t* in_, uint32_t len_, uint8_t* out, uint32_t out_lim) {
    in = in_;
    len = len_;
    pos = 0;
    size = 0;
    out0 = out;
    e.out = out;
    e.end = out + out_lim;
    e.low = 0;
    e.range = ~0u;
    m.reset();
  }

  // One input byte; true = the packet is finished and `size` holds compress()'s result.
  __host__ __device__ bool step(Model& m) {
    if (pos >= len) {  // :79-81 (one slice; a single empty slice codes nothing)
      size = 0;
      return true;
    }
    const uint32_t value = in[pos];
    uint32_t parent = ~0u;
    uint32_t ctx = m.predicted;
    bool coded = false;
    while (ctx != 0) {  // :130-297
      uint32_t under = 0, count = 0;
      const uint32_t sym = m.update(ctx, value, kSubSymbolDelta, under, count);
      m.set_parent(parent, sym);
      parent = sym;
      const Sym x = m.load(ctx);
      uint32_t total = lo16(x.w);
      uint32_t esc = hi16(x.z);
      if (count > 0) {
        if (!e.put(esc + under, count, total)) return fail();
      } else {
        if (esc > 0 && esc < total)
          if (!e.put(0, esc, total)) return fail();
        esc = (esc + kSubEscapeDelta) & 0xFFFF;
        total = (total + kSubEscapeDelta) & 0xFFFF;
        m.words(ctx)[2] = pack(x.z, esc);
      }
      total = (total + kSubSymbolDelta) & 0xFFFF;
      m.words(ctx)[3] = pack(total, hi16(x.w));
      if (count > 0xff - 2 * kSubSymbolDelta || total > kBottom - 0x100) m.ctx_rescale(ctx, 0);
      if (count > 0) {
        coded = true;
        break;
      }
      ctx = hi16(x.w);
    }
    if (!coded) {  // root, :298-420
      uint32_t under = value * kSymbolMinimum, count = kSymbolMinimum;
      const uint32_t sym = m.update(0, value, kCtxSymbolDelta, under, count);
      m.set_parent(parent, sym);
      const Sym r = m.load(0);
      if (!e.put(hi16(r.z) + under, count, lo16(r.w))) return fail();
      const uint32_t total = (lo16(r.w) + kCtxSymbolDelta) & 0xFFFF;
      m.words(0)[3] = pack(total, hi16(r.w));
      if (count > 0xff - 2 * kCtxSymbolDelta + kSymbolMinimum || total > kBottom - 0x100)
        m.ctx_rescale(0, 256 * kSymbolMinimum);
    }
    m.advance();
    if (++pos < len) return false;
    while (e.low) {  // :452-460
      if (e.out >= e.end) return fail();
      *e.out++ = (uint8_t)(e.low >> 24);
      e.low <<= 8;
    }
    size = (uint32_t)(e.out - out0);
    return true;
  }

  __host__ __device__ bool fail() {  // output limit reached: compress() returns 0
    size = 0;
    return true;
  }
};

[[maybe_unused]] __host__ __device__ uint32_t compress_one(Model& m, const uint8_t* in, uint32_t len, uint8_t* out, uint32_t out_lim) {
  if (len == 0) return 0;  // :79-81
  CompressLane c;
  c.begin(m, in, len, out, out_lim);
  while (!c.step(m)) {
  }
  return c.size;
}

struct Decoder {
  uint32_t low = 0, code = 0, range = ~0u;
  const uint8_t* in;
  const uint8_t* end;
  // decode renormalise, e.g. compress.rs:551-569
  RC_MODEL_ATTR __host__ __device__ void take(uint32_t under, uint32_t count) {
    low += under * range;
    range *= count;
    for (;;) {
      if ((low ^ (low + range)) >= kTop) {
        if (range >= kBottom) return;
        range = (0u - low) & (kBottom - 1);
      }
      code <<= 8;
      if (in < end) code |= *in++;
      range <<= 8;
      low <<= 8;
    }
  }
};

// enet_range_coder_decompress (compress.rs:463-987) as a resumable per-lane state
// machine (see CompressLane): step() decodes ONE symbol.
struct DecompressLane {
  Decoder d;
  uint8_t* out;
  uint32_t n, out_lim, size;
  bool empty;

  __host__ __device__ void begin(Model& m, const uint8_t* in, uint32_t len, uint8_t* out_, uint32_t out_lim_) {
    d.low = 0;
    d.code = 0;
    d.range = ~0u;
    d.in = in;
    d.end = in + len;
    out = out_;
    out_lim = out_lim_;
    n = 0;
    size = 0;
    empty = len == 0;  // :481-483
    m.reset();
    for (int k = 24; k >= 0; k -= 8)  // :500-519
      if (d.in < d.end) d.code |= (uint32_t)(*d.in++) << k;
  }

  __host__ __device__ bool finish(uint32_t result) {
    size = result;
    return true;
  }

  // One symbol; true = the packet is finished and `size` holds decompress()'s result.
  RC_DECODE_ATTR __host__ __device__ bool step(Model& m) {
    if (empty) return finish(0);
    uint32_t value = 0, bottom = 0;
    uint32_t ctx = m.predicted;
    bool found = false;
    while (ctx != 0) {  // :535-667
      const Sym x = m.load(ctx);
      const uint32_t esc = hi16(x.z), xtotal = lo16(x.w);
      if (esc > 0 && esc < xtotal) {
        d.range /= xtotal;
        uint32_t code = ((d.code - d.low) / d.range) & 0xFFFF;
        if (code < esc) {
          d.take(0, esc);
        } else {
          code = (code - esc) & 0xFFFF;
          uint32_t under = 0, count = 0;
          if (lo16(x.z) == 0) return finish(RC_FAIL(1, n));
          uint32_t i = ctx + lo16(x.z);
          for (;;) {  // :579-611
            const Sym s = m.load(i);
            const uint32_t su = hi16(s.x), sc = sym_count(s);
            const uint32_t after = (under + su) & 0xFFFF;
            if (code >= after) {
              under = after;
              if (!hi16(s.y)) return finish(RC_FAIL(2, n));
              i += hi16(s.y);
            } else if ((int)code < (int)after - (int)sc) {
              m.words(i)[0] = pack(s.x, su + kSubSymbolDelta);
              if (!lo16(s.y)) return finish(RC_FAIL(3, n));
              i += lo16(s.y);
            } else {
              value = sym_value(s);
              count = (count + sc) & 0xFFFF;
              under = (after - sc) & 0xFFFF;
              m.words(i)[0] = sym_x(value, sc + kSubSymbolDelta, (su + kSubSymbolDelta) & 0xFFFF);
              break;
            }
          }
          bottom = i;
          d.take(esc + under, count);
          const uint32_t total = (xtotal + kSubSymbolDelta) & 0xFFFF;
          m.words(ctx)[3] = pack(total, hi16(x.w));
          if (count > 0xff - 2 * kSubSymbolDelta || total > kBottom - 0x100) m.ctx_rescale(ctx, 0);
          found = true;
          break;
        }
      }
      ctx = hi16(x.w);
    }
    if (!found) {  // root, :668-840
      const Sym r = m.load(0);
      d.range /= lo16(r.w);
      uint32_t code = ((d.code - d.low) / d.range) & 0xFFFF;
      if (code < hi16(r.z)) {  // end of stream, :674-696
        d.take(0, hi16(r.z));
        size = n;
        return true;
      }
      code = (code - hi16(r.z)) & 0xFFFF;
      uint32_t under = 0, count = kSymbolMinimum, sym;
      if (lo16(r.z) == 0) {
        value = (code / kSymbolMinimum) & 0xFF;
        under = (code - code % kSymbolMinimum) & 0xFFFF;
        sym = m.new_symbol(value, kCtxSymbolDelta);
        m.words(0)[2] = pack(sym, hi16(r.z));
      } else {
        uint32_t i = lo16(r.z);
        for (;;) {  // :719-796
          const Sym s = m.load(i);
          const uint32_t su = hi16(s.x), sc = sym_count(s), sv = sym_value(s);
          const int after = (int)((under + su + (sv + 1u) * kSymbolMinimum) & 0xFFFF);
          const int before = (int)((sc + kSymbolMinimum) & 0xFFFF);
          const int c = (int)code;
          if (c >= after) {
            under = (under + su) & 0xFFFF;
            if (hi16(s.y)) {
              i += hi16(s.y);
              continue;
            }
            value = (uint32_t)((int)sv + 1 + (c - after) / (int)kSymbolMinimum) & 0xFF;
            under = (uint32_t)(c - (c - after) % (int)kSymbolMinimum) & 0xFFFF;
            sym = m.new_symbol(value, kCtxSymbolDelta);
            m.words(i)[1] = pack(s.y, sym - i);
            break;
          }
          if (c < after - before) {
            m.words(i)[0] = pack(s.x, su + kCtxSymbolDelta);
            if (lo16(s.y)) {
              i += lo16(s.y);
              continue;
            }
            value = (uint32_t)((int)sv - 1 - (after - before - c - 1) / (int)kSymbolMinimum) & 0xFF;
            under = (uint32_t)(c - (after - before - c - 1) % (int)kSymbolMinimum) & 0xFFFF;
            sym = m.new_symbol(value, kCtxSymbolDelta);
            m.words(i)[1] = pack(sym - i, hi16(s.y));
            break;
          }
          value = sv;
          count = (count + sc) & 0xFFFF;
          under = (uint32_t)(after - before) & 0xFFFF;
          m.words(i)[0] = sym_x(sv, sc + kCtxSymbolDelta, (su + kCtxSymbolDelta) & 0xFFFF);
          sym = i;
          break;
        }
      }
      bottom = sym;
      const Sym r2 = m.load(0);
      d.take(hi16(r2.z) + under, count);
      const uint32_t total = (lo16(r2.w) + kCtxSymbolDelta) & 0xFFFF;
      m.words(0)[3] = pack(total, hi16(r2.w));
      if (count > 0xff - 2 * kCtxSymbolDelta + kSymbolMinimum || total > kBottom - 0x100)
        m.ctx_rescale(0, 256 * kSymbolMinimum);
    }
    // patch the higher-order contexts, :841-948
    uint32_t parent = ~0u;
    for (uint32_t p = m.predicted; p != ctx;) {
      uint32_t under = 0, count = 0;
      const uint32_t sym = m.update(p, value, kSubSymbolDelta, under, count);
      m.set_parent(parent, sym);
      parent = sym;
      const Sym x = m.load(p);
      uint32_t total = lo16(x.w);
      if (count == 0) {
        m.words(p)[2] = pack(x.z, hi16(x.z) + kSubEscapeDelta);
        total = (total + kSubEscapeDelta) & 0xFFFF;
      }
      total = (total + kSubSymbolDelta) & 0xFFFF;
      m.words(p)[3] = pack(total, hi16(x.w));
      if (count > 0xff - 2 * kSubSymbolDelta || total > kBottom - 0x100) m.ctx_rescale(p, 0);
      p = hi16(x.w);
    }
    m.set_parent(parent, bottom);
    if (n >= out_lim) return finish(RC_FAIL(4, n));  // :949-954
    out[n++] = (uint8_t)value;
    m.advance();
    return false;
  }
};

[[maybe_unused]] RC_DECODE_ATTR __host__ __device__ uint32_t decompress_one(Model& m, const uint8_t* in, uint32_t len, uint8_t* out,
                                                           uint32_t out_lim) {
  if (len == 0) return 0;  // :481-483
  DecompressLane dl;
  dl.begin(m, in, len, out, out_lim);
  while (!dl.step(m)) {
  }
  return dl.size;
}

struct RangeBatch {
  const uint8_t* in;
  const uint64_t* in_off;
  const uint32_t* in_len;
  uint64_t count;
  uint8_t* out;
  const uint64_t* out_off;
  const uint32_t* out_lim;
  uint32_t* sizes;
  Sym* arenas;
  uint64_t workers;
};

// One lane = one coder: packets w, w + workers, ... in turn, one symbol per loop trip;
// a lane whose packet finishes starts its next one on the next trip.
template <bool kDecompress>
__global__ __launch_bounds__(kBlock) void range_coder_kernel(RangeBatch b) {
  const uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (w >= b.workers || w >= b.count) return;
  Model m;
  m.a = b.arenas + w * kArena;
  m.next = 0;
  m.predicted = 0;
  m.order = 0;
  using Lane = typename std::conditional<kDecompress, DecompressLane, CompressLane>::type;
  Lane lane;
  uint64_t p = w;
  lane.begin(m, b.in + b.in_off[p], b.in_len[p], b.out + b.out_off[p], b.out_lim[p]);
  for (;;) {
    if (lane.step(m)) {
      b.sizes[p] = lane.size;
      p += b.workers;
      if (p >= b.count) break;
      lane.begin(m, b.in + b.in_off[p], b.in_len[p], b.out + b.out_off[p], b.out_lim[p]);
    }
  }
}

}  // namespace

hipError_t launch_range(bool decompress, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                        uint64_t count, uint8_t* out, const uint64_t* out_off, const uint32_t* out_lim,
                        uint32_t* sizes, void* scratch, uint64_t workers, hipStream_t stream) {
  if (count == 0) return hipSuccess;
  if (workers > count) workers = count;
  if (workers == 0) return hipErrorInvalidValue;
  RangeBatch b{in, in_off, in_len, count, out, out_off, out_lim, sizes, static_cast<Sym*>(scratch), workers};
  const dim3 grid((unsigned)((workers + kBlock - 1) / kBlock));
  if (decompress)
    hipLaunchKernelGGL(range_coder_kernel<true>, grid, dim3(kBlock), 0, stream, b);
  else
    hipLaunchKernelGGL(range_coder_kernel<false>, grid, dim3(kBlock), 0, stream, b);
  return hipGetLastError();
}

}  // namespace enet_crc
