// gfx950 kernels of the ENet range coder: the `Compressor`
// implementation `RangeCoder` of jabuwu/rusty_enet (src/compressor.rs:36-69) over
// src/c/compress.rs, batched across packets.
//
// The coder is sequential inside a packet (every symbol updates the adaptive
// order-2 model that codes the next one), so the parallelism is across packets:
// one lane = one coder = one packet at a time (grid-stride over the batch).
// Each lane owns a 64 KiB symbol arena (4096 x 16-B ENetSymbol, compress.rs:7-22)
// in HBM scratch.  A symbol is read as ONE 16-byte load; updates are narrow
// stores to the fields that change.  The work is a chain of dependent arena
// loads (tree walks in up to three contexts per byte), so the kernel is
// latency-bound, not bandwidth-bound: throughput comes from the number of lanes
// in flight (the `workers` argument sizes the scratch and the grid).
//
// Semantics follow compress.rs statement for statement (line numbers below),
// including the u16/u8 wrap-around of every counter and the arena reset at
// 4094 symbols (:426-450).
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// decompress_one is built without optimisation: at -O1 and above the gfx950 build of
// its body decodes wrong symbols after a few steps, while the host build of the same
// source is bit-exact (tools/dbg/standalone.hip).  The Model methods it
// calls stay optimised.
#ifndef RC_DECODE_ATTR
#define RC_DECODE_ATTR __attribute__((optnone))
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

struct alignas(16) Sym {  // ENetSymbol, compress.rs:12-22 (same 16-B layout)
  uint8_t value;
  uint8_t count;
  uint16_t under;
  uint16_t left;
  uint16_t right;
  uint16_t symbols;
  uint16_t escapes;
  uint16_t total;
  uint16_t parent;
};
static_assert(sizeof(Sym) == 16, "ENetSymbol is 16 bytes");
static_assert(kArena * sizeof(Sym) == kRangeArenaBytes, "arena size");

struct Model {
  Sym* a;
  uint32_t next;
  uint32_t predicted;
  uint32_t order;

  __host__ __device__ Sym load(uint32_t i) const { return a[i]; }

  RC_MODEL_ATTR __host__ __device__ uint32_t new_symbol(uint32_t value, uint32_t delta) {
    const uint32_t i = next++;
    Sym s{};
    s.value = (uint8_t)value;
    s.count = (uint8_t)delta;
    s.under = (uint16_t)delta;
    a[i] = s;
    return i;
  }

  // compress.rs:86-101 / :426-450
  RC_MODEL_ATTR __host__ __device__ void reset() {
    Sym r{};
    r.escapes = kEscapeMinimum;
    r.total = kEscapeMinimum + 256 * kSymbolMinimum;
    a[0] = r;
    next = 1;
    predicted = 0;
    order = 0;
  }

  // `parent` chain target: ~0u = the `predicted` register, else the .parent field of a symbol.
  RC_MODEL_ATTR __host__ __device__ void set_parent(uint32_t slot, uint32_t v) {
    if (slot == ~0u)
      predicted = v;
    else
      a[slot].parent = (uint16_t)v;
  }

  // enet_symbol_rescale, compress.rs:42-59, with the left recursion on an explicit
  // stack (a context tree has at most 256 nodes).  Stack entry = node | frame total << 16.
  RC_MODEL_ATTR __host__ __device__ uint32_t rescale(uint32_t i) {
    uint32_t stk[256];
    int sp = 0;
    uint32_t total = 0;
    for (;;) {
      Sym s = load(i);
      s.count = (uint8_t)(s.count - (s.count >> 1));
      a[i].count = s.count;
      a[i].under = s.count;
      if (s.left) {  // descend; finish this node after the left subtree returns
        stk[sp++] = i | (total << 16);
        i += s.left;
        total = 0;
        continue;
      }
      total = (total + s.count) & 0xFFFF;
      // walk right; when a frame ends, return its total to the node that pushed it
      for (;;) {
        if (s.right) {
          i += s.right;
          break;
        }
        if (sp == 0) return total;
        const uint32_t e = stk[--sp];
        const uint32_t sub = total;
        i = e & 0xFFFF;
        total = e >> 16;
        const uint16_t u = (uint16_t)(a[i].under + sub);
        a[i].under = u;
        total = (total + u) & 0xFFFF;
        s = load(i);
      }
    }
  }

  // find-or-insert `value` in context ctx's tree (compress.rs:137-212, :301-376, :847-922).
  RC_MODEL_ATTR __host__ __device__ uint32_t update(uint32_t ctx, uint32_t value, uint32_t delta, uint32_t& under, uint32_t& count) {
    const uint32_t first = a[ctx].symbols;
    if (first == 0) {
      const uint32_t n = new_symbol(value, delta);
      a[ctx].symbols = (uint16_t)(n - ctx);
      return n;
    }
    uint32_t i = ctx + first;
    for (;;) {
      const Sym s = load(i);
      if (value < s.value) {
        a[i].under = (uint16_t)(s.under + delta);
        if (s.left) {
          i += s.left;
          continue;
        }
        const uint32_t n = new_symbol(value, delta);
        a[i].left = (uint16_t)(n - i);
        return n;
      }
      if (value > s.value) {
        under = (under + s.under) & 0xFFFF;
        if (s.right) {
          i += s.right;
          continue;
        }
        const uint32_t n = new_symbol(value, delta);
        a[i].right = (uint16_t)(n - i);
        return n;
      }
      count = (count + s.count) & 0xFFFF;
      under = (under + (uint32_t)s.under - s.count) & 0xFFFF;
      a[i].under = (uint16_t)(s.under + delta);
      a[i].count = (uint8_t)(s.count + delta);
      return i;
    }
  }

  // :276-289
  RC_MODEL_ATTR __host__ __device__ void sub_rescale(uint32_t ctx) {
    const uint32_t sy = a[ctx].symbols;
    uint32_t t = sy ? rescale(ctx + sy) : 0;
    const uint16_t esc = a[ctx].escapes;
    const uint16_t e2 = (uint16_t)(esc - (esc >> 1));
    a[ctx].escapes = e2;
    a[ctx].total = (uint16_t)(t + e2);
  }

  // :404-419
  RC_MODEL_ATTR __host__ __device__ void root_rescale() {
    const uint32_t sy = a[0].symbols;
    uint32_t t = sy ? rescale(sy) : 0;
    const uint16_t esc = a[0].escapes;
    const uint16_t e2 = (uint16_t)(esc - (esc >> 1));
    a[0].escapes = e2;
    a[0].total = (uint16_t)(t + e2 + 256 * kSymbolMinimum);
  }

  // :421-450, after every symbol
  RC_MODEL_ATTR __host__ __device__ void advance() {
    if (order >= kOrder)
      predicted = a[predicted].parent;
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

// enet_range_coder_compress over one contiguous input (compress.rs:60-462).
__host__ __device__ uint32_t compress_one(Model& m, const uint8_t* in, uint32_t len, uint8_t* out, uint32_t out_lim) {
  if (len == 0) return 0;  // :79-81 (one slice; a single empty slice codes nothing)
  Encoder e;
  e.out = out;
  e.end = out + out_lim;
  m.reset();
  uint32_t nextv = in[0];
  for (uint32_t pos = 0; pos < len; ++pos) {
    const uint32_t value = nextv;
    if (pos + 1 < len) nextv = in[pos + 1];  // issue the next byte's load early
    uint32_t parent = ~0u;
    uint32_t ctx = m.predicted;
    bool coded = false;
    while (ctx != 0) {  // :130-297
      uint32_t under = 0, count = 0;
      const uint32_t sym = m.update(ctx, value, kSubSymbolDelta, under, count);
      m.set_parent(parent, sym);
      parent = sym;
      const Sym x = m.load(ctx);
      uint32_t total = x.total;
      uint32_t esc = x.escapes;
      if (count > 0) {
        if (!e.put(esc + under, count, total)) return 0;
      } else {
        if (esc > 0 && esc < total)
          if (!e.put(0, esc, total)) return 0;
        esc = (esc + kSubEscapeDelta) & 0xFFFF;
        total = (total + kSubEscapeDelta) & 0xFFFF;
        m.a[ctx].escapes = (uint16_t)esc;
      }
      total = (total + kSubSymbolDelta) & 0xFFFF;
      m.a[ctx].total = (uint16_t)total;
      if (count > 0xff - 2 * kSubSymbolDelta || total > kBottom - 0x100) m.sub_rescale(ctx);
      if (count > 0) {
        coded = true;
        break;
      }
      ctx = x.parent;
    }
    if (!coded) {  // root, :298-420
      uint32_t under = value * kSymbolMinimum, count = kSymbolMinimum;
      const uint32_t sym = m.update(0, value, kCtxSymbolDelta, under, count);
      m.set_parent(parent, sym);
      const Sym r = m.load(0);
      if (!e.put((uint32_t)r.escapes + under, count, r.total)) return 0;
      const uint32_t total = (r.total + kCtxSymbolDelta) & 0xFFFF;
      m.a[0].total = (uint16_t)total;
      if (count > 0xff - 2 * kCtxSymbolDelta + kSymbolMinimum || total > kBottom - 0x100) m.root_rescale();
    }
    m.advance();
  }
  while (e.low) {  // :452-460
    if (e.out >= e.end) return 0;
    *e.out++ = (uint8_t)(e.low >> 24);
    e.low <<= 8;
  }
  return (uint32_t)(e.out - out);
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

// enet_range_coder_decompress (compress.rs:463-987).
RC_DECODE_ATTR __host__ __device__ uint32_t decompress_one(Model& m, const uint8_t* in, uint32_t len, uint8_t* out, uint32_t out_lim) {
  if (len == 0) return 0;  // :481-483
  Decoder d;
  d.in = in;
  d.end = in + len;
  m.reset();
  for (int k = 24; k >= 0; k -= 8)  // :500-519
    if (d.in < d.end) d.code |= (uint32_t)(*d.in++) << k;
  uint32_t n = 0;
  for (;;) {
    uint32_t value = 0, bottom = 0;
    uint32_t ctx = m.predicted;
    bool found = false;
    while (ctx != 0) {  // :535-667
      const Sym x = m.load(ctx);
      if (x.escapes > 0 && x.escapes < x.total) {
        d.range /= x.total;
        uint32_t code = ((d.code - d.low) / d.range) & 0xFFFF;
        if (code < x.escapes) {
          d.take(0, x.escapes);
        } else {
          code = (code - x.escapes) & 0xFFFF;
          uint32_t under = 0, count = 0;
          if (x.symbols == 0) return RC_FAIL(1, n);
          uint32_t i = ctx + x.symbols;
          for (;;) {  // :579-611
            const Sym s = m.load(i);
            const uint32_t after = (under + s.under) & 0xFFFF;
            const uint32_t before = s.count;
            if (code >= after) {
              under = (under + s.under) & 0xFFFF;
              if (!s.right) return RC_FAIL(2, n);
              i += s.right;
            } else if ((int)code < (int)after - (int)before) {
              m.a[i].under = (uint16_t)(s.under + kSubSymbolDelta);
              if (!s.left) return RC_FAIL(3, n);
              i += s.left;
            } else {
              value = s.value;
              count = (count + s.count) & 0xFFFF;
              under = (after - before) & 0xFFFF;
              m.a[i].under = (uint16_t)(s.under + kSubSymbolDelta);
              m.a[i].count = (uint8_t)(s.count + kSubSymbolDelta);
              break;
            }
          }
          bottom = i;
          d.take((uint32_t)x.escapes + under, count);
          const uint32_t total = (x.total + kSubSymbolDelta) & 0xFFFF;
          m.a[ctx].total = (uint16_t)total;
          if (count > 0xff - 2 * kSubSymbolDelta || total > kBottom - 0x100) m.sub_rescale(ctx);
          found = true;
          break;
        }
      }
      ctx = x.parent;
    }
    if (!found) {  // root, :668-840
      const Sym r = m.load(0);
      d.range /= r.total;
      uint32_t code = ((d.code - d.low) / d.range) & 0xFFFF;
      if (code < r.escapes) {  // end of stream, :674-696
        d.take(0, r.escapes);
        break;
      }
      code = (code - r.escapes) & 0xFFFF;
      uint32_t under = 0, count = kSymbolMinimum, sym;
      if (r.symbols == 0) {
        value = (code / kSymbolMinimum) & 0xFF;
        under = (code - code % kSymbolMinimum) & 0xFFFF;
        sym = m.new_symbol(value, kCtxSymbolDelta);
        m.a[0].symbols = (uint16_t)sym;
      } else {
        uint32_t i = r.symbols;
        for (;;) {  // :719-796
          const Sym s = m.load(i);
          const int after = (int)((under + s.under + (s.value + 1u) * kSymbolMinimum) & 0xFFFF);
          const int before = (int)((s.count + kSymbolMinimum) & 0xFFFF);
          const int c = (int)code;
          if (c >= after) {
            under = (under + s.under) & 0xFFFF;
            if (s.right) {
              i += s.right;
              continue;
            }
            value = (uint32_t)(s.value + 1 + (c - after) / (int)kSymbolMinimum) & 0xFF;
            under = (uint32_t)(c - (c - after) % (int)kSymbolMinimum) & 0xFFFF;
            sym = m.new_symbol(value, kCtxSymbolDelta);
            m.a[i].right = (uint16_t)(sym - i);
            break;
          }
          if (c < after - before) {
            m.a[i].under = (uint16_t)(s.under + kCtxSymbolDelta);
            if (s.left) {
              i += s.left;
              continue;
            }
            value = (uint32_t)(s.value - 1 - (after - before - c - 1) / (int)kSymbolMinimum) & 0xFF;
            under = (uint32_t)(c - (after - before - c - 1) % (int)kSymbolMinimum) & 0xFFFF;
            sym = m.new_symbol(value, kCtxSymbolDelta);
            m.a[i].left = (uint16_t)(sym - i);
            break;
          }
          value = s.value;
          count = (count + s.count) & 0xFFFF;
          under = (uint32_t)(after - before) & 0xFFFF;
          m.a[i].under = (uint16_t)(s.under + kCtxSymbolDelta);
          m.a[i].count = (uint8_t)(s.count + kCtxSymbolDelta);
          sym = i;
          break;
        }
      }
      bottom = sym;
      const Sym r2 = m.load(0);
      d.take((uint32_t)r2.escapes + under, count);
      const uint32_t total = (r2.total + kCtxSymbolDelta) & 0xFFFF;
      m.a[0].total = (uint16_t)total;
      if (count > 0xff - 2 * kCtxSymbolDelta + kSymbolMinimum || total > kBottom - 0x100) m.root_rescale();
    }
    // patch the higher-order contexts, :841-948
    uint32_t parent = ~0u;
    for (uint32_t p = m.predicted; p != ctx;) {
      uint32_t under = 0, count = 0;
      const uint32_t sym = m.update(p, value, kSubSymbolDelta, under, count);
      m.set_parent(parent, sym);
      parent = sym;
      const Sym x = m.load(p);
      uint32_t total = x.total;
      if (count == 0) {
        m.a[p].escapes = (uint16_t)(x.escapes + kSubEscapeDelta);
        total = (total + kSubEscapeDelta) & 0xFFFF;
      }
      total = (total + kSubSymbolDelta) & 0xFFFF;
      m.a[p].total = (uint16_t)total;
      if (count > 0xff - 2 * kSubSymbolDelta || total > kBottom - 0x100) m.sub_rescale(p);
      p = x.parent;
    }
    m.set_parent(parent, bottom);
#ifdef RC_DEBUG_EXITS
    if (2048 + 16 * (n + 1) <= out_lim) {  // debug trace: per symbol, after the patch loop
      uint32_t* t = (uint32_t*)(out + 2048 + 16 * n);
      t[0] = value | (ctx << 8) | (m.predicted << 20);
      t[1] = d.low;
      t[2] = d.range;
      t[3] = d.code;
    }
    if (n == 3 && out_lim >= 4096 + 256) {  // debug: arena[0..15] after symbol 3
      for (int k = 0; k < 16; ++k) *(Sym*)(out + 4096 + 16 * k) = m.a[k];
    }
#endif
    if (n >= out_lim) return RC_FAIL(4, n);  // :949-954
    out[n++] = (uint8_t)value;
    m.advance();
  }
  return n;
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

template <bool kDecompress>
__global__ __launch_bounds__(kBlock) void range_coder_kernel(RangeBatch b) {
  const uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (w >= b.workers) return;
  Model m;
  m.a = b.arenas + w * kArena;
  m.next = 0;
  m.predicted = 0;
  m.order = 0;
  for (uint64_t p = w; p < b.count; p += b.workers) {
    const uint8_t* in = b.in + b.in_off[p];
    uint8_t* out = b.out + b.out_off[p];
    const uint32_t len = b.in_len[p], lim = b.out_lim[p];
    b.sizes[p] = kDecompress ? decompress_one(m, in, len, out, lim) : compress_one(m, in, len, out, lim);
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
