/*
 * enet_crc_amd.h -- C ABI of the MI355X (gfx950) ENet CRC-32 checksum path.
 *
 * Drop-in for the checksum hook of jabuwu/rusty_enet v0.4.0:
 *   - src/crc32.rs:39   pub fn crc32(in_buffers: &[&[u8]]) -> u32
 *   - src/host.rs:40    HostSettings::checksum: Option<Box<dyn Fn(&[&[u8]]) -> u32>>
 *   - src/c/protocol.rs:1470-1502 (receive verify) and :2255-2293 (send insert),
 *     the two call sites of that hook.
 *
 * Every checksum this library returns equals the reference's value for the
 * same bytes: bswap32(~reg) of the reflected-0xEDB88320 register started at
 * 0xFFFFFFFF over the CONCATENATION of the input slices (src/crc32.rs:40-46).
 *
 * Conventions
 *   - Plain C types only; the caller owns every buffer.
 *   - Functions return an int status (ENET_CRC_OK = 0, negative on error).
 *     Nothing here falls back to the CPU: without a usable HIP device the
 *     calls fail with ENET_CRC_E_NO_DEVICE / ENET_CRC_E_HIP.
 *   - "*_device" functions take device pointers and a hipStream_t passed as
 *     void* (NULL = the legacy default stream); they are asynchronous and
 *     run on the calling thread's current HIP device.
 *     (An explicit stream's own device is used, whatever device is current.)
 *   - A context (enet_crc_ctx) owns, per entry of its device list, a stream pair
 *     plus pinned/device staging for the host-memory entry points.  Calls on
 *     one context are serialised by an internal lock, which is what lets the
 *     Rust adapter present it as the `Fn` (not `FnMut`) closure
 *     HostSettings::checksum requires.
 */
#ifndef ENET_CRC_AMD_H
#define ENET_CRC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ENET_CRC_ABI_VERSION 6

#if defined(__GNUC__)
#define ENET_CRC_API __attribute__((visibility("default")))
#else
#define ENET_CRC_API
#endif

#define ENET_CRC_OK 0
#define ENET_CRC_E_INVALID (-1)   /* bad argument (NULL pointer, count overflow) */
#define ENET_CRC_E_NO_DEVICE (-2) /* no HIP device / bad device index */
#define ENET_CRC_E_HIP (-3)       /* a HIP runtime call failed; see enet_crc_last_hip_error() */
#define ENET_CRC_E_NOMEM (-4)     /* host or device allocation failed */
/* A batch kernel gave up on the device (an inter-wave wait of the ragged kernel timed out):
 * the batch's outputs are invalid.  See enet_crc_device_status(). */
#define ENET_CRC_E_DEVICE (-5)

/* Shape of ENetBuffer {data, data_length} (src/c.rs:25-28): one input slice. */
typedef struct enet_crc_iov {
  const uint8_t* data;
  size_t len;
} enet_crc_iov;

typedef struct enet_crc_ctx enet_crc_ctx;

/* Most entries in a context's device list. */
#define ENET_CRC_MAX_LANES 64

/*
 * Per-call modes of enet_crc32_iov (enet_crc_ctx_set_percall_mode).
 *
 * Where the per-call hook stands.  One datagram per call cannot beat the CPU it
 * replaces: src/crc32.rs runs a 1392-B datagram in ~2.2 us on one host core, while the
 * fastest GPU mode below costs ~3.4 us from C, of which the PCIe round
 * trip alone (host store -> GPU -> host) is ~1.7 us.  Installing enet_crc32_iov as
 * HostSettings::checksum therefore slows every datagram.  The GPU pays off on batches:
 * the batched receive verify / send insert below (INTEGRATION.md §3 is the recommended
 * integration), at ~5 TB/s on the device.
 */
#define ENET_CRC_PERCALL_COPY 0     /* pinned staging -> H2D copy -> kernel -> D2H copy (~24 us) */
/* (default) One single-packet launch that reads the gathered bytes from mapped pinned
 * memory and writes the result to mapped memory; nothing stays resident (~21 us through
 * ctypes on the round-4 box). */
#define ENET_CRC_PERCALL_ZEROCOPY 1
/* Opt-in.  A server wave stays resident on lane 0's device and polls a request mailbox
 * (device memory the host writes through the PCIe BAR on large-BAR devices, else pinned
 * host memory; answers in pinned host memory): no kernel launch per call (~3.4 us).
 * Datagrams above 4096 B take the zero-copy path.  While it runs:
 *   - any batch launch on that device (any context, the context-free *_device entry points,
 *     rings) sends it home first: it exits at its next poll, so the batch gets every CU, and
 *     the next per-call call relaunches it (one launch, ~20-40 us);
 *   - a device-wide synchronisation (hipDeviceSynchronize, torch.cuda.synchronize())
 *     waits for it: it exits 20 ms after the last call, or at once on
 *     enet_crc_ctx_stop_server(), a mode change, a batch entry of the same context or
 *     enet_crc_ctx_destroy;
 *   - a call the server does not answer within 5 s stops it, returns ENET_CRC_E_HIP
 *     (hipErrorLaunchTimeOut) and switches the context back to ZEROCOPY. */
#define ENET_CRC_PERCALL_PERSISTENT 2

/* ENET_CRC_ABI_VERSION: 4 added enet_crc32_combine; 5 added enet_crc_ctx_percall_mode and
 * enet_crc_ctx_stop_server and made ZEROCOPY the default per-call mode; 6 added
 * ENET_CRC_E_DEVICE and enet_crc_device_status.  Nothing was removed.  Behaviour changes
 * within ABI 6: enet_crc32_shards_device checks placement and rejects buffers that are not
 * device memory of the shard's device (mapped pinned host memory and managed memory, which
 * it used to read over the fabric, now return ENET_CRC_E_INVALID); enet_crc_ctx_stop_server
 * returns ENET_CRC_E_HIP (hipErrorLaunchTimeOut) when the server wave does not stop; the
 * synchronous entries report only their own launches' failures (per-slot failure words)
 * and no longer read or clear the device word. */
ENET_CRC_API int enet_crc_abi_version(void);
ENET_CRC_API const char* enet_crc_strerror(int status);
/* hipError_t of the last failing HIP call made by this thread (0 if none). */
ENET_CRC_API int enet_crc_last_hip_error(void);
/* Number of visible HIP devices (0 when none), or a negative status. */
ENET_CRC_API int enet_crc_device_count(void);

/*
 * Device-side failure channel.  The ragged batch kernel synchronises its waves through
 * flags in LDS; a wait that does not complete within its poll limit (never observed:
 * DESIGN.md §4) is given up rather than left to hang the GPU.  The wave that gives up
 * writes a failure bit (1: a job's records never became ready, 2: a job slot was never
 * released, 4: a result slot was never flushed) into the failure word its launch carries,
 * and its workgroup stops writing checksums.  Words are sticky until cleared:
 *   - the synchronous entries (enet_crc32_ragged_host, enet_crc_ring_wait, and the
 *     receive/send loops built on them) give every staging / ring slot a word of its own,
 *     cleared before the slot's launches and read after the call's last wait: such a call
 *     returns ENET_CRC_E_DEVICE exactly when one of its own launches failed (no output of
 *     that call may be trusted), whatever else runs on the device;
 *   - the asynchronous *_device entries report into the device's word: synchronise the
 *     stream and call enet_crc_device_status(device, clear): > 0 means some asynchronous
 *     batch on that device since the last clear produced invalid outputs (the word is
 *     shared by every asynchronous caller on the device).
 * Returns the bits (0 = no failure), or a negative status for a bad device.
 */
ENET_CRC_API int enet_crc_device_status(int device, int clear);

/* Create a context bound to HIP device `device` (its own non-blocking streams,
 * pinned + device staging grown on demand).  Same as
 * enet_crc_ctx_create_multi(&device, 1, out_ctx). */
ENET_CRC_API int enet_crc_ctx_create(int device, enet_crc_ctx** out_ctx);

/*
 * Create a context over a device list (the batch split across the
 * GPUs of one node).  Entry i is a "lane": device devices[i] with its own stream
 * pair, staging and (for i >= 1) host worker thread.  A device may appear more than
 * once (two lanes on one GPU).  enet_crc32_ragged_host on such a context splits the
 * batch into ndevices byte-balanced contiguous shards (enet_crc_shard_bounds) and
 * checksums shard i on lane i, all lanes at once; the per-call and range-coder entry
 * points use lane 0.  1 <= ndevices <= ENET_CRC_MAX_LANES.
 */
ENET_CRC_API int enet_crc_ctx_create_multi(const int* devices, uint32_t ndevices, enet_crc_ctx** out_ctx);
ENET_CRC_API void enet_crc_ctx_destroy(enet_crc_ctx* ctx);
/* Number of lanes (device-list entries) of a context, or ENET_CRC_E_INVALID. */
ENET_CRC_API int enet_crc_ctx_lanes(const enet_crc_ctx* ctx);
/* Select how enet_crc32_iov moves one datagram (ENET_CRC_PERCALL_*; default ZEROCOPY). */
ENET_CRC_API int enet_crc_ctx_set_percall_mode(enet_crc_ctx* ctx, int mode);
/* The context's current per-call mode (ENET_CRC_PERCALL_*), or ENET_CRC_E_INVALID. */
ENET_CRC_API int enet_crc_ctx_percall_mode(enet_crc_ctx* ctx);
/* Stop the context's persistent server wave now, if one runs (the next persistent-mode
 * call relaunches it).  Call before a device-wide synchronisation.  ENET_CRC_E_HIP
 * (hipErrorLaunchTimeOut) if the wave ignored the request for 3 s (it still holds a CU
 * until its 2-s lifetime ends; batch entries still run, one workgroup starting late). */
ENET_CRC_API int enet_crc_ctx_stop_server(enet_crc_ctx* ctx);

/*
 * Byte-balanced contiguous split of a batch into `nshards` packet ranges:
 * bounds[0] = 0 <= bounds[1] <= ... <= bounds[nshards] = count; shard k is packets
 * [bounds[k], bounds[k+1]).  Cut k is one past the first packet whose cumulative
 * byte end reaches floor(total_bytes * k / nshards), so every shard is within one
 * packet of total/nshards bytes.  lengths == NULL: an even split by packet count.
 * Host function, no device work.
 */
ENET_CRC_API int enet_crc_shard_bounds(const uint32_t* lengths, uint64_t count, uint32_t nshards,
                                       uint64_t* bounds);

/*
 * Per-call drop-in for `crc32(in_buffers)` (src/crc32.rs:39-47).
 * Replaces: the closure stored in HostSettings::checksum (src/host.rs:40) and
 * called at src/c/protocol.rs:1499 (one slice) and :2287 (up to 65 slices,
 * BUFFER_MAXIMUM, src/consts.rs:37).  Slices may be empty or NULL-with-len-0.
 * Gathers the slices into pinned memory, checksums on the GPU, writes the reference
 * value to *out_crc.  Synchronous.  How the bytes move: the context's per-call mode
 * (ENET_CRC_PERCALL_*, default ZEROCOPY).  Slower than the CPU per datagram (see the
 * modes above); batch instead where the protocol loop allows it.
 */
ENET_CRC_API int enet_crc32_iov(enet_crc_ctx* ctx, const enet_crc_iov* bufs, size_t nbufs, uint32_t* out_crc);

/*
 * Device-resident uniform batch: packet p is the `length` bytes at
 * d_base + p*stride, p in [0, count).  d_out[p] = crc32(&[packet p]).
 * Replaces `count` calls of src/crc32.rs:39 with one launch.
 */
ENET_CRC_API int enet_crc32_uniform_device(const void* d_base, uint64_t stride, uint32_t length, uint64_t count,
                              uint32_t* d_out, void* hip_stream);

/*
 * Device-resident ragged batch: packet p is d_lengths[p] bytes at
 * d_base + d_offsets[p] (any byte alignment, packed or not).
 */
ENET_CRC_API int enet_crc32_ragged_device(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                             uint64_t count, uint32_t* d_out, void* hip_stream);

/*
 * Device-resident batch sharded over several devices: shard i is a uniform
 * (d_offsets == NULL: packets at d_base + p*stride, `length` bytes) or ragged
 * (d_offsets/d_lengths) batch in device `device`'s memory, checksummed on that
 * device into d_out on hip_stream (a stream of that device, or NULL).  Every
 * launch is asynchronous (nothing waits: synchronise each shard's stream); the shards
 * run concurrently on their devices.  Placement is checked before anything launches:
 * d_base, d_out, d_offsets and d_lengths must be device memory of `device` and
 * hip_stream a stream of `device`, else ENET_CRC_E_INVALID and no shard runs.
 */
typedef struct enet_crc_shard {
  int device;
  const void* d_base;
  const uint64_t* d_offsets; /* NULL: uniform shard */
  const uint32_t* d_lengths;
  uint64_t stride;
  uint32_t length;
  uint64_t count;
  uint32_t* d_out;
  void* hip_stream;
} enet_crc_shard;

ENET_CRC_API int enet_crc32_shards_device(const enet_crc_shard* shards, size_t nshards);

/*
 * Host-resident ragged batch (the end-to-end path: host packet buffers such as
 * the UdpSocket receive buffers of src/c/protocol.rs:1660-1680 in, checksums
 * out).  Stages through pinned memory in chunks, overlapping copy and compute
 * on the context's stream pair.  On a multi-device context the batch is split into
 * one byte-balanced shard per lane and the lanes run concurrently; outputs go to
 * disjoint slices of h_out.  Synchronous.  On an error no later write into h_out
 * happens (everything in flight is waited for first).
 */
ENET_CRC_API int enet_crc32_ragged_host(enet_crc_ctx* ctx, const void* h_base, const uint64_t* h_offsets,
                           const uint32_t* h_lengths, uint64_t count, uint32_t* h_out);

/*
 * Batched receive verify.  Replaces, for `count` received
 * datagrams, the per-datagram check of src/c/protocol.rs:1470-1502: read the u32 in
 * the 4-byte checksum slot at d_slot_offsets[p] (header_size - 4, :1470-1478),
 * overwrite it with d_slot_values[p] (peer.connect_id, or 0 for peer id 4095,
 * :1483-1492), checksum the datagram (:1493-1499) and accept it when the two match.
 * Datagram p is d_lengths[p] bytes at d_base + d_offsets[p] (as received, i.e. after
 * any decompression, :1455-1468).  Outputs: d_crc[p] = the checksum the reference
 * computes at :1499; d_ok[p] = 1 (accept) or 0 (drop, :1499-1501; also when the slot
 * does not fit inside the datagram).  The datagram bytes are NOT modified.  The slot
 * value is applied by linearity after the checksum pass, so the GPU never writes the
 * buffers.  Device pointers, asynchronous on `hip_stream`.
 */
ENET_CRC_API int enet_crc32_verify_ragged_device(const void* d_base, const uint64_t* d_offsets,
                                                 const uint32_t* d_lengths, const uint32_t* d_slot_offsets,
                                                 const uint32_t* d_slot_values, uint64_t count, uint32_t* d_crc,
                                                 uint32_t* d_ok, void* hip_stream);

/*
 * Batched send insert.  Replaces, for `count` assembled outgoing
 * datagrams, src/c/protocol.rs:2255-2293: the slot at d_slot_offsets[p] takes
 * d_slot_values[p] (connect_id, or 0 while outgoing_peer_id >= 4095, :2259-2266),
 * the datagram is checksummed (:2276-2286) and the checksum is written into the slot
 * native-endian (:2287-2292).  d_crc[p] receives the checksum too.  Datagrams are
 * contiguous (header, slot, then the commands) and must not overlap.  A slot that
 * does not fit inside its datagram is left untouched (d_crc[p] = checksum as stored).
 */
ENET_CRC_API int enet_crc32_insert_ragged_device(void* d_base, const uint64_t* d_offsets, const uint32_t* d_lengths,
                                                 const uint32_t* d_slot_offsets, const uint32_t* d_slot_values,
                                                 uint64_t count, uint32_t* d_crc, void* hip_stream);

/*
 * Host-side slot correction (no device work; O(log n) table steps).  Given the
 * checksum `crc` of a datagram whose slot holds `old_slot`, returns the checksum of
 * the same datagram with the slot holding `new_slot`, where `bytes_after_slot` bytes
 * follow the slot.  This is what lets a receive loop checksum a whole batch before it
 * knows each datagram's connect_id: an earlier CONNECT in the same batch can change
 * it (src/c/protocol.rs:550), and the reference reads it at processing time (:1483).
 */
ENET_CRC_API uint32_t enet_crc32_slot_adjust(uint32_t crc, uint32_t old_slot, uint32_t new_slot,
                                             uint32_t bytes_after_slot);

/*
 * Host-side merge (no device work; O(log len_b) table steps; GF(2) matrix squarings past 16 GiB).  Given the
 * checksums crc_a = crc32(&[a]) and crc_b = crc32(&[b]) in the reference's convention
 * (src/crc32.rs:46, bswap32(~reg)), returns crc32(&[a, b]), the checksum of the
 * concatenation, where len_b is the byte length of b (any u64).  This is the merged
 * digest of a sharded batch: per-shard or per-packet checksums
 * computed on different GPUs combine on the host without touching the bytes again.
 * len_b == 0 returns crc_a.
 */
ENET_CRC_API uint32_t enet_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/*
 * Pinned receive ring.  The host path above copies pageable
 * buffers into pinned staging first; a ring lets the receive loop put datagrams
 * straight into pinned memory (e.g. recvmmsg into slot memory, the role of
 * host->packet_data in src/c/protocol.rs:1660-1665) and overlaps each slot's
 * H2D copy, checksum kernel and D2H copy with the other slots'.
 *
 * A ring has `nslots` slots on device `device`; each slot owns a pinned byte buffer
 * of `slot_bytes`, pinned descriptor arrays for `slot_packets` packets (u64 offsets
 * into the slot's bytes, u32 lengths), a pinned result array, device mirrors and its
 * own stream.  enet_crc_ring_slot() returns the host pointers (any may be NULL).
 * enet_crc_ring_submit(ring, i, count) queues H2D -> checksum -> D2H for packets
 * 0..count-1 of slot i and returns at once; the slot's memory must not be touched
 * until enet_crc_ring_wait(ring, i) has returned, after which crcs[0..count) hold the
 * reference checksums.  Submitting a slot that is in flight is ENET_CRC_E_INVALID,
 * as is a packet outside the slot's bytes.  Calls on one ring are thread-safe.
 * The status of a wait belongs to the slot's last submit: ENET_CRC_E_DEVICE as long as
 * that submit's launch gave up on the device (every later wait on the slot says so too,
 * until the next submit), else ENET_CRC_OK.
 */
typedef struct enet_crc_ring enet_crc_ring;

ENET_CRC_API int enet_crc_ring_create(int device, uint32_t nslots, uint64_t slot_bytes, uint32_t slot_packets,
                                      enet_crc_ring** out_ring);
ENET_CRC_API void enet_crc_ring_destroy(enet_crc_ring* ring);
ENET_CRC_API int enet_crc_ring_slot(enet_crc_ring* ring, uint32_t slot, uint8_t** data, uint64_t** offsets,
                                    uint32_t** lengths, uint32_t** crcs);
ENET_CRC_API int enet_crc_ring_submit(enet_crc_ring* ring, uint32_t slot, uint64_t count);
ENET_CRC_API int enet_crc_ring_wait(enet_crc_ring* ring, uint32_t slot);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* ENET_CRC_AMD_H */
