/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by or called
 * from the product library (rusty_enet_amd/).  Only tests/, the smoke() check
 * in __graft_entry__.py and bench.py's cpu_baseline leg use it, and only as the
 * checker / CPU baseline.
 *
 * A plain-C restatement of jabuwu/rusty_enet v0.4.0 src/crc32.rs (the Rust
 * reference cannot be built here: no cargo/rustc in the image, so there is no
 * oracle/_ref).  Pinned by:
 *   - the reference's own known-answer tests, src/crc32.rs:49-57
 *     ([1..8] -> 3314076223; [1..8] ++ [8..1] as two slices -> 1712484799),
 *   - the JSON fixtures under tests/golden, generated with Python's zlib (an independent CRC-32
 *     implementation; reference value = bswap32(zlib.crc32(concat))),
 *   checked in tests/test_oracle.py.
 *
 * Also restates the ENet checksum-slot conventions of src/c/protocol.rs
 * (receive verify :1470-1502, send insert :2255-2293) for the protocol-level
 * parity tests.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

/* src/crc32.rs:1-34 CRC_TABLE: the reflected 0xEDB88320 table, generated here
 * bit by bit rather than copied. */
static uint32_t g_table[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void build_table(void) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t r = b;
    for (int i = 0; i < 8; ++i) r = (r & 1u) ? (r >> 1) ^ 0xEDB88320u : (r >> 1);
    g_table[b] = r;
  }
}

static inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

typedef struct oracle_iov {
  const uint8_t* data;
  size_t len;
} oracle_iov;

const uint32_t* oracle_crc_table(void) {
  pthread_once(&g_once, build_table);
  return g_table;
}

/* Register-level helpers (no init, no finalisation). */
uint32_t oracle_crc_update(uint32_t crc, const uint8_t* p, size_t n) {
  pthread_once(&g_once, build_table);
  for (size_t i = 0; i < n; ++i) crc = (crc >> 8) ^ g_table[(crc & 0xFFu) ^ (uint32_t)p[i]]; /* :43 */
  return crc;
}

/* src/crc32.rs:39-47  pub fn crc32(in_buffers: &[&[u8]]) -> u32 */
uint32_t oracle_crc32_iov(const oracle_iov* bufs, size_t n) {
  uint32_t crc = 0xFFFFFFFFu;                                  /* :40 */
  for (size_t i = 0; i < n; ++i) crc = oracle_crc_update(crc, bufs[i].data, bufs[i].len); /* :41-45 */
  return bswap32(~crc);                                        /* :46 (!crc).to_be() on LE */
}

uint32_t oracle_crc32(const uint8_t* p, size_t n) {
  oracle_iov one = {p, n};
  return oracle_crc32_iov(&one, 1);
}

/* One call per packet, as the reference's Host does (single slice, :1493-1499). */
void oracle_crc32_ragged(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                         uint64_t count, uint32_t* out) {
  for (uint64_t i = 0; i < count; ++i) out[i] = oracle_crc32(base + offsets[i], lengths[i]);
}

void oracle_crc32_uniform(const uint8_t* base, uint64_t stride, uint32_t length, uint64_t count,
                          uint32_t* out) {
  for (uint64_t i = 0; i < count; ++i) out[i] = oracle_crc32(base + i * stride, length);
}

/* Multi-threaded drivers (packet range split): the all-cores CPU baseline, and the
 * checker for full-size GPU batches.  offsets == NULL: uniform packets at i * stride. */
typedef struct {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint32_t* lengths;
  uint64_t stride;
  uint32_t length;
  uint64_t first, last;
  uint32_t* out;
} mt_job;

static void* mt_worker(void* arg) {
  mt_job* j = (mt_job*)arg;
  for (uint64_t i = j->first; i < j->last; ++i)
    j->out[i] = j->offsets ? oracle_crc32(j->base + j->offsets[i], j->lengths[i])
                           : oracle_crc32(j->base + i * j->stride, j->length);
  return NULL;
}

static int run_mt(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths, uint64_t stride,
                  uint32_t length, uint64_t count, uint32_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  mt_job jobs[256];
  pthread_once(&g_once, build_table);
  int started = 0, rc = 0;
  for (int t = 0; t < threads; ++t) {
    jobs[t].base = base;
    jobs[t].offsets = offsets;
    jobs[t].lengths = lengths;
    jobs[t].stride = stride;
    jobs[t].length = length;
    jobs[t].first = count * (uint64_t)t / (uint64_t)threads;
    jobs[t].last = count * (uint64_t)(t + 1) / (uint64_t)threads;
    jobs[t].out = out;
    if (pthread_create(&tid[t], NULL, mt_worker, &jobs[t]) != 0) {
      rc = -1;
      break;
    }
    ++started;
  }
  for (int t = 0; t < started; ++t) pthread_join(tid[t], NULL);
  return rc;
}

int oracle_crc32_uniform_mt(const uint8_t* base, uint64_t stride, uint32_t length, uint64_t count,
                            uint32_t* out, int threads) {
  return run_mt(base, NULL, NULL, stride, length, count, out, threads);
}

int oracle_crc32_ragged_mt(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths, uint64_t count,
                           uint32_t* out, int threads) {
  return run_mt(base, offsets, lengths, 0, 0, count, out, threads);
}

/*
 * ENet receive verify, src/c/protocol.rs:1412-1415 + 1470-1502, restated.
 *   header_size = (sent_time flag ? 4 : 2) + 4; the 4 bytes ending at
 *   header_size hold the sender's checksum (native-endian u32 read, :1473-1478);
 *   they are overwritten with `slot_value` (peer.connect_id, or 0 when the
 *   peer id is PROTOCOL_MAXIMUM_PEER_ID, :1483-1492) and the whole datagram is
 *   checksummed as ONE slice (:1493-1499).  Returns 1 if the datagram is
 *   accepted, 0 if it would be dropped.  `datagram` is modified exactly like
 *   the reference modifies host->received_data.
 */
int oracle_enet_verify(uint8_t* datagram, size_t length, size_t header_size, uint32_t slot_value) {
  if (header_size < 4 || header_size > length) return 0;
  uint8_t* slot = datagram + header_size - 4;
  uint32_t desired;
  memcpy(&desired, slot, 4);
  memcpy(slot, &slot_value, 4);
  return oracle_crc32(datagram, length) == desired;
}

/*
 * ENet send insert, src/c/protocol.rs:2255-2293, restated for the common
 * scatter list: buffers[0] is the header (2 or 4 bytes) and is extended by the
 * 4-byte slot, which first holds `slot_value` (connect_id, or 0 while
 * outgoing_peer_id >= PROTOCOL_MAXIMUM_PEER_ID); the checksum of
 * header||slot||buffers[1..] (UNcompressed, :2294-2299 swap happens after) is
 * then written into the slot native-endian.  `header` must have room for
 * header_len + 4 bytes.  Returns the checksum.
 */
uint32_t oracle_enet_insert(uint8_t* header, size_t header_len, const oracle_iov* rest, size_t nrest,
                            uint32_t slot_value) {
  memcpy(header + header_len, &slot_value, 4);
  uint32_t crc = 0xFFFFFFFFu;
  crc = oracle_crc_update(crc, header, header_len + 4);
  for (size_t i = 0; i < nrest; ++i) crc = oracle_crc_update(crc, rest[i].data, rest[i].len);
  uint32_t out = bswap32(~crc);
  memcpy(header + header_len, &out, 4);
  return out;
}
