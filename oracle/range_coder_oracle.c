/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by or called
 * from the product library (rusty_enet_amd/).  Only tests/ and bench.py's
 * cpu_baseline leg use it, as the checker / CPU baseline.
 *
 * Plain-C restatement of the ENet range coder of jabuwu/rusty_enet v0.4.0,
 * src/c/compress.rs (the `Compressor` implementation `RangeCoder`,
 * src/compressor.rs:36-69): an adaptive order-2 context model whose contexts are
 * the 4096-entry symbol arena (compress.rs:7-22), coded with a carry-less range
 * coder (TOP = 2^24, BOTTOM = 2^16, compress.rs:23-30).
 *
 * Parity status: the reference has no tests or fixtures for the range coder and
 * cannot be built here (no rustc), so this restatement is pinned only by
 * (a) following compress.rs statement by statement (line numbers below) and
 * (b) the round-trip property decompress(compress(x)) == x, checked in
 * tests/test_range_oracle.py over random, low-entropy, multi-slice and reset-
 * crossing inputs.  "Parity unpinned" by reference vectors.
 *
 * Input-slice rule (compress.rs:110-126): the coder reads the first slice, then
 * moves to the next slice only when the current one is exhausted, one slice per
 * symbol step.  An EMPTY slice reached that way is read as one 0 byte: Rust
 * empty slices carry the dangling pointer (c.rs:79-85), which compress.rs:119-122
 * turns into a 0 symbol.  An empty FIRST slice contributes nothing.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

enum {
  SYMBOL_MINIMUM = 1,     /* compress.rs:23 */
  ESCAPE_MINIMUM = 1,     /* :24 */
  SUBCONTEXT_ORDER = 2,   /* :25 */
  RC_BOTTOM = 65536,      /* :26 */
  SUB_SYMBOL_DELTA = 2,   /* :27 */
  SUB_ESCAPE_DELTA = 5,   /* :28 */
  CTX_SYMBOL_DELTA = 3,   /* :29 */
  RC_TOP = 16777216,      /* :30 */
  ARENA = 4096            /* :8 */
};

typedef struct osym { /* ENetSymbol, compress.rs:12-22 */
  uint8_t value, count;
  uint16_t under, left, right, symbols, escapes, total, parent;
} osym;

typedef struct ocoder {
  osym s[ARENA];
  size_t next;
} ocoder;

typedef struct oracle_iov {
  const uint8_t* data;
  size_t len;
} oracle_iov;

static uint16_t new_symbol(ocoder* c, uint8_t value, uint8_t delta) {
  size_t i = c->next++;
  osym* s = &c->s[i];
  memset(s, 0, sizeof *s);
  s->value = value;
  s->count = delta;
  s->under = delta;
  return (uint16_t)i;
}

/* root (re)initialisation, compress.rs:86-101 and :426-450 */
static void reset_root(ocoder* c) {
  c->next = 0;
  size_t r = c->next++;
  memset(&c->s[r], 0, sizeof c->s[r]);
  c->s[r].escapes = ESCAPE_MINIMUM;
  c->s[r].total = ESCAPE_MINIMUM + 256 * SYMBOL_MINIMUM;
}

/* enet_symbol_rescale, compress.rs:42-59 (left recursion, right iteration) */
static uint16_t rescale(ocoder* c, size_t i) {
  uint16_t total = 0;
  for (;;) {
    osym* s = &c->s[i];
    s->count = (uint8_t)(s->count - (s->count >> 1));
    s->under = s->count;
    if (s->left) s->under = (uint16_t)(s->under + rescale(c, i + s->left));
    total = (uint16_t)(total + s->under);
    if (!s->right) break;
    i += s->right;
  }
  return total;
}

/* Tree update by value inside context `ctx` (compress.rs:137-212 with delta 2,
 * :301-376 with delta 3, decompress patch :847-922): find or insert `value`,
 * accumulating the cumulative frequency below it into *under and its count
 * into *count.  Returns the arena index of the symbol. */
static uint16_t update_by_value(ocoder* c, size_t ctx, uint8_t value, uint8_t delta, uint16_t* under,
                                uint16_t* count) {
  if (c->s[ctx].symbols == 0) {
    uint16_t n = new_symbol(c, value, delta);
    c->s[ctx].symbols = (uint16_t)(n - ctx);
    return n;
  }
  size_t i = ctx + c->s[ctx].symbols;
  for (;;) {
    osym* s = &c->s[i];
    if (value < s->value) {
      s->under = (uint16_t)(s->under + delta);
      if (s->left) { i += s->left; continue; }
      uint16_t n = new_symbol(c, value, delta);
      c->s[i].left = (uint16_t)(n - i);
      return n;
    } else if (value > s->value) {
      *under = (uint16_t)(*under + s->under);
      if (s->right) { i += s->right; continue; }
      uint16_t n = new_symbol(c, value, delta);
      c->s[i].right = (uint16_t)(n - i);
      return n;
    } else {
      *count = (uint16_t)(*count + s->count);
      *under = (uint16_t)(*under + (s->under - s->count));
      s->under = (uint16_t)(s->under + delta);
      s->count = (uint8_t)(s->count + delta);
      return (uint16_t)i;
    }
  }
}

/* ---------------------------------------------------------------- encoder */

typedef struct enc {
  uint32_t low, range;
  uint8_t* out;
  uint8_t* end;
} enc;

/* the encode + renormalise blocks, e.g. compress.rs:217-241 */
static int enc_put(enc* e, uint32_t under, uint32_t count, uint32_t total) {
  e->range /= total;
  e->low += under * e->range;
  e->range *= count;
  for (;;) {
    if ((e->low ^ (e->low + e->range)) >= RC_TOP) {
      if (e->range >= RC_BOTTOM) break;
      e->range = (0u - e->low) & (RC_BOTTOM - 1);
    }
    if (e->out >= e->end) return 0;
    *e->out++ = (uint8_t)(e->low >> 24);
    e->range <<= 8;
    e->low <<= 8;
  }
  return 1;
}

/* subcontext / root rescale triggers, compress.rs:276-289 and :404-419 */
static void sub_rescale(ocoder* c, size_t ctx) {
  osym* x = &c->s[ctx];
  x->total = x->symbols ? rescale(c, ctx + x->symbols) : 0;
  x->escapes = (uint16_t)(x->escapes - (x->escapes >> 1));
  x->total = (uint16_t)(x->total + x->escapes);
}

static void root_rescale(ocoder* c) {
  osym* r = &c->s[0];
  r->total = r->symbols ? rescale(c, r->symbols) : 0;
  r->escapes = (uint16_t)(r->escapes - (r->escapes >> 1));
  r->total = (uint16_t)(r->total + r->escapes + 256 * SYMBOL_MINIMUM);
}

/* enet_range_coder_compress, compress.rs:60-462.  Returns the compressed size,
 * 0 when the output would exceed out_limit or the input is empty. */
size_t oracle_range_compress(const oracle_iov* bufs, size_t nbufs, size_t in_limit, uint8_t* out,
                             size_t out_limit) {
  static __thread ocoder c;
  if (nbufs == 0 || in_limit == 0) return 0; /* :79-81 */
  enc e = {0u, ~0u, out, out + out_limit};
  const uint8_t* in = bufs[0].data;
  size_t left = bufs[0].len, bi = 1;
  int dangling = 0;
  uint16_t predicted = 0;
  size_t order = 0;
  reset_root(&c);
  for (;;) {
    uint8_t value;
    if (left == 0 && !dangling) { /* :110-118 */
      if (bi >= nbufs) break;
      in = bufs[bi].data;
      left = bufs[bi].len;
      ++bi;
      if (left == 0) dangling = 1;
    }
    if (dangling) { /* :119-122 */
      value = 0;
      dangling = 0;
    } else {
      value = *in++;
      --left;
    }
    uint16_t* parent = &predicted;
    size_t ctx = predicted;
    int coded = 0;
    while (ctx != 0) { /* :130-297 */
      uint16_t under = 0, count = 0;
      uint16_t sym = update_by_value(&c, ctx, value, SUB_SYMBOL_DELTA, &under, &count);
      *parent = sym;
      parent = &c.s[sym].parent;
      osym* x = &c.s[ctx];
      uint16_t total = x->total;
      if (count > 0) {
        if (!enc_put(&e, (uint32_t)x->escapes + under, count, total)) return 0;
      } else {
        if (x->escapes > 0 && x->escapes < total)
          if (!enc_put(&e, 0, x->escapes, total)) return 0;
        x->escapes = (uint16_t)(x->escapes + SUB_ESCAPE_DELTA);
        x->total = (uint16_t)(x->total + SUB_ESCAPE_DELTA);
      }
      x->total = (uint16_t)(x->total + SUB_SYMBOL_DELTA);
      if (count > 0xff - 2 * SUB_SYMBOL_DELTA || x->total > RC_BOTTOM - 0x100) sub_rescale(&c, ctx);
      if (count > 0) { coded = 1; break; }
      ctx = x->parent;
    }
    if (!coded) { /* root, :298-420 */
      uint16_t under = (uint16_t)(value * SYMBOL_MINIMUM), count = SYMBOL_MINIMUM;
      uint16_t sym = update_by_value(&c, 0, value, CTX_SYMBOL_DELTA, &under, &count);
      *parent = sym;
      osym* r = &c.s[0];
      if (!enc_put(&e, (uint32_t)r->escapes + under, count, r->total)) return 0;
      r->total = (uint16_t)(r->total + CTX_SYMBOL_DELTA);
      if (count > 0xff - 2 * CTX_SYMBOL_DELTA + SYMBOL_MINIMUM || r->total > RC_BOTTOM - 0x100) root_rescale(&c);
    }
    if (order >= SUBCONTEXT_ORDER) /* :421-425 */
      predicted = c.s[predicted].parent;
    else
      ++order;
    if (c.next >= ARENA - SUBCONTEXT_ORDER) { /* :426-450 */
      reset_root(&c);
      predicted = 0;
      order = 0;
    }
  }
  while (e.low) { /* :452-460 */
    if (e.out >= e.end) return 0;
    *e.out++ = (uint8_t)(e.low >> 24);
    e.low <<= 8;
  }
  return (size_t)(e.out - out);
}

/* ---------------------------------------------------------------- decoder */

typedef struct dec {
  uint32_t low, code, range;
  const uint8_t* in;
  const uint8_t* end;
} dec;

/* decode renormalise blocks, e.g. compress.rs:551-569 */
static void dec_take(dec* d, uint32_t under, uint32_t count) {
  d->low += under * d->range;
  d->range *= count;
  for (;;) {
    if ((d->low ^ (d->low + d->range)) >= RC_TOP) {
      if (d->range >= RC_BOTTOM) break;
      d->range = (0u - d->low) & (RC_BOTTOM - 1);
    }
    d->code <<= 8;
    if (d->in < d->end) d->code |= *d->in++;
    d->range <<= 8;
    d->low <<= 8;
  }
}

/* enet_range_coder_decompress, compress.rs:463-987.  Returns the decompressed
 * size, 0 on a malformed stream or when out_limit is reached. */
size_t oracle_range_decompress(const uint8_t* in, size_t in_len, uint8_t* out, size_t out_limit) {
  static __thread ocoder c;
  if (in_len == 0) return 0; /* :481-483 */
  uint8_t* o = out;
  uint8_t* oend = out + out_limit;
  dec d = {0u, 0u, ~0u, in, in + in_len};
  uint16_t predicted = 0;
  size_t order = 0;
  reset_root(&c);
  for (int k = 24; k >= 0; k -= 8) /* :500-519 */
    if (d.in < d.end) d.code |= (uint32_t)(*d.in++) << k;
  for (;;) {
    uint8_t value = 0;
    uint16_t bottom = 0;
    uint16_t* parent = &predicted;
    size_t ctx = predicted;
    int found = 0;
    while (ctx != 0) { /* :535-667 */
      osym* x = &c.s[ctx];
      if (x->escapes > 0) {
        uint16_t total = x->total;
        if (x->escapes < total) {
          d.range /= total;
          uint16_t code = (uint16_t)((d.code - d.low) / d.range);
          if (code < x->escapes) {
            dec_take(&d, 0, x->escapes);
          } else {
            code = (uint16_t)(code - x->escapes);
            uint16_t under = 0, count = 0;
            if (x->symbols == 0) return 0;
            size_t i = ctx + x->symbols;
            for (;;) { /* :579-611 */
              osym* s = &c.s[i];
              uint16_t after = (uint16_t)(under + s->under);
              uint16_t before = s->count;
              if (code >= after) {
                under = (uint16_t)(under + s->under);
                if (!s->right) return 0;
                i += s->right;
              } else if (code < after - before) {
                s->under = (uint16_t)(s->under + SUB_SYMBOL_DELTA);
                if (!s->left) return 0;
                i += s->left;
              } else {
                value = s->value;
                count = (uint16_t)(count + s->count);
                under = (uint16_t)(after - before);
                s->under = (uint16_t)(s->under + SUB_SYMBOL_DELTA);
                s->count = (uint8_t)(s->count + SUB_SYMBOL_DELTA);
                break;
              }
            }
            bottom = (uint16_t)i;
            dec_take(&d, (uint32_t)x->escapes + under, count);
            x->total = (uint16_t)(x->total + SUB_SYMBOL_DELTA);
            if (count > 0xff - 2 * SUB_SYMBOL_DELTA || x->total > RC_BOTTOM - 0x100) sub_rescale(&c, ctx);
            found = 1;
            break;
          }
        }
      }
      ctx = x->parent;
    }
    if (!found) { /* root, :668-840 */
      osym* r = &c.s[0];
      d.range /= r->total;
      uint16_t code = (uint16_t)((d.code - d.low) / d.range);
      if (code < r->escapes) { /* end of stream, :674-696 */
        dec_take(&d, 0, r->escapes);
        break;
      }
      code = (uint16_t)(code - r->escapes);
      uint16_t under = 0, count = SYMBOL_MINIMUM;
      uint16_t sym;
      if (r->symbols == 0) {
        value = (uint8_t)(code / SYMBOL_MINIMUM);
        under = (uint16_t)(code - code % SYMBOL_MINIMUM);
        sym = new_symbol(&c, value, CTX_SYMBOL_DELTA);
        c.s[0].symbols = sym;
      } else {
        size_t i = r->symbols;
        for (;;) { /* :719-796 */
          osym* s = &c.s[i];
          int after = (uint16_t)(under + s->under + (s->value + 1) * SYMBOL_MINIMUM);
          int before = (uint16_t)(s->count + SYMBOL_MINIMUM);
          if (code >= after) {
            under = (uint16_t)(under + s->under);
            if (s->right) { i += s->right; continue; }
            value = (uint8_t)(s->value + 1 + (code - after) / SYMBOL_MINIMUM);
            under = (uint16_t)(code - (code - after) % SYMBOL_MINIMUM);
            sym = new_symbol(&c, value, CTX_SYMBOL_DELTA);
            c.s[i].right = (uint16_t)(sym - i);
            break;
          } else if (code < after - before) {
            s->under = (uint16_t)(s->under + CTX_SYMBOL_DELTA);
            if (s->left) { i += s->left; continue; }
            value = (uint8_t)(s->value - 1 - (after - before - code - 1) / SYMBOL_MINIMUM);
            under = (uint16_t)(code - (after - before - code - 1) % SYMBOL_MINIMUM);
            sym = new_symbol(&c, value, CTX_SYMBOL_DELTA);
            c.s[i].left = (uint16_t)(sym - i);
            break;
          } else {
            value = s->value;
            count = (uint16_t)(count + s->count);
            under = (uint16_t)(after - before);
            s->under = (uint16_t)(s->under + CTX_SYMBOL_DELTA);
            s->count = (uint8_t)(s->count + CTX_SYMBOL_DELTA);
            sym = (uint16_t)i;
            break;
          }
        }
      }
      bottom = sym;
      r = &c.s[0];
      dec_take(&d, (uint32_t)r->escapes + under, count);
      r->total = (uint16_t)(r->total + CTX_SYMBOL_DELTA);
      if (count > 0xff - 2 * CTX_SYMBOL_DELTA + SYMBOL_MINIMUM || r->total > RC_BOTTOM - 0x100) root_rescale(&c);
    }
    /* patch the contexts above the one that coded the symbol, :841-948 */
    for (size_t p = predicted; p != ctx;) {
      uint16_t under = 0, count = 0;
      uint16_t sym = update_by_value(&c, p, value, SUB_SYMBOL_DELTA, &under, &count);
      *parent = sym;
      parent = &c.s[sym].parent;
      osym* x = &c.s[p];
      if (count == 0) {
        x->escapes = (uint16_t)(x->escapes + SUB_ESCAPE_DELTA);
        x->total = (uint16_t)(x->total + SUB_ESCAPE_DELTA);
      }
      x->total = (uint16_t)(x->total + SUB_SYMBOL_DELTA);
      if (count > 0xff - 2 * SUB_SYMBOL_DELTA || x->total > RC_BOTTOM - 0x100) sub_rescale(&c, p);
      p = x->parent;
    }
    *parent = bottom;
    if (o >= oend) return 0; /* :949-954 */
    *o++ = value;
    if (order >= SUBCONTEXT_ORDER) /* :955-959 */
      predicted = c.s[predicted].parent;
    else
      ++order;
    if (c.next >= ARENA - SUBCONTEXT_ORDER) { /* :960-984 */
      reset_root(&c);
      predicted = 0;
      order = 0;
    }
  }
  return (size_t)(o - out);
}

/* Batched helpers for the parity tests / CPU baseline: packet p is in_len[p]
 * bytes at in + in_off[p]; its output goes to out + out_off[p] (limit
 * out_lim[p]); the returned size goes to sizes[p]. */
void oracle_range_compress_ragged(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint64_t n,
                                  uint8_t* out, const uint64_t* out_off, const uint32_t* out_lim, uint32_t* sizes) {
  for (uint64_t p = 0; p < n; ++p) {
    oracle_iov one = {in + in_off[p], in_len[p]};
    sizes[p] = (uint32_t)oracle_range_compress(&one, 1, in_len[p], out + out_off[p], out_lim[p]);
  }
}

void oracle_range_decompress_ragged(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint64_t n,
                                    uint8_t* out, const uint64_t* out_off, const uint32_t* out_lim, uint32_t* sizes) {
  for (uint64_t p = 0; p < n; ++p)
    sizes[p] = (uint32_t)oracle_range_decompress(in + in_off[p], in_len[p], out + out_off[p], out_lim[p]);
}
