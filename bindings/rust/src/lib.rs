//! Rust side of the drop-in: binds `include/enet_crc_amd.h` and produces the
//! closure `rusty_enet::HostSettings::checksum` expects
//! (`Option<Box<dyn Fn(&[&[u8]]) -> u32>>`, rusty_enet src/host.rs:40).
//!
//! ```ignore
//! let gpu = enet_crc_amd::GpuCrc32::new(0)?;
//! let settings = rusty_enet::HostSettings {
//!     checksum: Some(gpu.checksum_fn()),   // was: Some(Box::new(rusty_enet::crc32))
//!     ..Default::default()
//! };
//! ```
//!
//! Written against the C ABI only; this image has no Rust toolchain, so the
//! crate is compiled where `cargo` exists.
#![allow(non_camel_case_types)]

use core::ffi::{c_int, c_void};
use std::sync::Arc;

#[repr(C)]
pub struct enet_crc_iov {
    pub data: *const u8,
    pub len: usize,
}

#[repr(C)]
pub struct enet_crc_ctx {
    _private: [u8; 0],
}

pub const ENET_CRC_OK: c_int = 0;
/// A batch kernel gave up on the device: the call's outputs are invalid (ABI 6).
pub const ENET_CRC_E_DEVICE: c_int = -5;
pub const ENET_CRC_PERCALL_COPY: c_int = 0;
pub const ENET_CRC_PERCALL_ZEROCOPY: c_int = 1;
pub const ENET_CRC_PERCALL_PERSISTENT: c_int = 2;

/// `enet_crc_shard` (include/enet_crc_amd.h): one device-resident batch of a
/// multi-device launch.  `d_offsets == null` means a uniform shard.
#[repr(C)]
pub struct enet_crc_shard {
    pub device: c_int,
    pub d_base: *const c_void,
    pub d_offsets: *const u64,
    pub d_lengths: *const u32,
    pub stride: u64,
    pub length: u32,
    pub count: u64,
    pub d_out: *mut u32,
    pub hip_stream: *mut c_void,
}

extern "C" {
    pub fn enet_crc_abi_version() -> c_int;
    pub fn enet_crc_strerror(status: c_int) -> *const core::ffi::c_char;
    pub fn enet_crc_last_hip_error() -> c_int;
    pub fn enet_crc_device_count() -> c_int;
    /// Device-side failure channel (ABI 6): > 0 if a batch kernel on `device` gave up since
    /// the last clear (its outputs are invalid); the synchronous entries return
    /// ENET_CRC_E_DEVICE (-5) instead.
    pub fn enet_crc_device_status(device: c_int, clear: c_int) -> c_int;
    pub fn enet_crc_ctx_create(device: c_int, out_ctx: *mut *mut enet_crc_ctx) -> c_int;
    pub fn enet_crc_ctx_create_multi(devices: *const c_int, ndevices: u32, out_ctx: *mut *mut enet_crc_ctx) -> c_int;
    pub fn enet_crc_ctx_destroy(ctx: *mut enet_crc_ctx);
    pub fn enet_crc_ctx_lanes(ctx: *const enet_crc_ctx) -> c_int;
    pub fn enet_crc_ctx_set_percall_mode(ctx: *mut enet_crc_ctx, mode: c_int) -> c_int;
    pub fn enet_crc_ctx_percall_mode(ctx: *mut enet_crc_ctx) -> c_int;
    pub fn enet_crc_ctx_stop_server(ctx: *mut enet_crc_ctx) -> c_int;
    pub fn enet_crc_shard_bounds(lengths: *const u32, count: u64, nshards: u32, bounds: *mut u64) -> c_int;
    pub fn enet_crc32_shards_device(shards: *const enet_crc_shard, nshards: usize) -> c_int;
    pub fn enet_crc32_iov(ctx: *mut enet_crc_ctx, bufs: *const enet_crc_iov, nbufs: usize, out_crc: *mut u32) -> c_int;
    pub fn enet_crc32_uniform_device(d_base: *const c_void, stride: u64, length: u32, count: u64,
                                     d_out: *mut u32, hip_stream: *mut c_void) -> c_int;
    pub fn enet_crc32_ragged_device(d_base: *const c_void, d_offsets: *const u64, d_lengths: *const u32,
                                    count: u64, d_out: *mut u32, hip_stream: *mut c_void) -> c_int;
    pub fn enet_crc32_ragged_host(ctx: *mut enet_crc_ctx, h_base: *const c_void, h_offsets: *const u64,
                                  h_lengths: *const u32, count: u64, h_out: *mut u32) -> c_int;
    pub fn enet_crc32_verify_ragged_device(d_base: *const c_void, d_offsets: *const u64, d_lengths: *const u32,
                                           d_slot_offsets: *const u32, d_slot_values: *const u32, count: u64,
                                           d_crc: *mut u32, d_ok: *mut u32, hip_stream: *mut c_void) -> c_int;
    pub fn enet_crc32_insert_ragged_device(d_base: *mut c_void, d_offsets: *const u64, d_lengths: *const u32,
                                           d_slot_offsets: *const u32, d_slot_values: *const u32, count: u64,
                                           d_crc: *mut u32, hip_stream: *mut c_void) -> c_int;
    pub fn enet_crc32_slot_adjust(crc: u32, old_slot: u32, new_slot: u32, bytes_after_slot: u32) -> u32;
    pub fn enet_crc32_combine(crc_a: u32, crc_b: u32, len_b: u64) -> u32;

    // include/enet_range_amd.h
    pub fn enet_range_scratch_bytes(workers: u64) -> u64;
    pub fn enet_range_compress_iov(ctx: *mut enet_crc_ctx, bufs: *const enet_crc_iov, nbufs: usize, in_limit: usize,
                                   out: *mut u8, out_limit: usize, out_size: *mut usize) -> c_int;
    pub fn enet_range_decompress(ctx: *mut enet_crc_ctx, input: *const u8, in_len: usize, out: *mut u8,
                                 out_limit: usize, out_size: *mut usize) -> c_int;
    pub fn enet_range_compress_ragged_host(ctx: *mut enet_crc_ctx, h_in: *const c_void, h_in_offsets: *const u64,
                                           h_in_lengths: *const u32, count: u64, h_out: *mut c_void,
                                           h_out_offsets: *const u64, h_out_limits: *const u32,
                                           h_sizes: *mut u32) -> c_int;
    pub fn enet_range_decompress_ragged_host(ctx: *mut enet_crc_ctx, h_in: *const c_void, h_in_offsets: *const u64,
                                             h_in_lengths: *const u32, count: u64, h_out: *mut c_void,
                                             h_out_offsets: *const u64, h_out_limits: *const u32,
                                             h_sizes: *mut u32) -> c_int;
    pub fn enet_range_compress_ragged_device(d_in: *const c_void, d_in_offsets: *const u64,
                                             d_in_lengths: *const u32, count: u64, d_out: *mut c_void,
                                             d_out_offsets: *const u64, d_out_limits: *const u32, d_sizes: *mut u32,
                                             d_scratch: *mut c_void, scratch_bytes: u64,
                                             hip_stream: *mut c_void) -> c_int;
    pub fn enet_range_decompress_ragged_device(d_in: *const c_void, d_in_offsets: *const u64,
                                               d_in_lengths: *const u32, count: u64, d_out: *mut c_void,
                                               d_out_offsets: *const u64, d_out_limits: *const u32,
                                               d_sizes: *mut u32, d_scratch: *mut c_void, scratch_bytes: u64,
                                               hip_stream: *mut c_void) -> c_int;
}

fn last_error(status: c_int) -> CrcError {
    CrcError { status, hip_error: unsafe { enet_crc_last_hip_error() } }
}

/// Checksum of a datagram after its 4-byte checksum slot changes from `old_slot` to
/// `new_slot` (`bytes_after_slot` bytes follow the slot).  Host-only; lets a receive
/// loop checksum a whole batch on the GPU first and apply each datagram's connect_id
/// when it processes the datagram (rusty_enet src/c/protocol.rs:1483-1499).
pub fn slot_adjust(crc: u32, old_slot: u32, new_slot: u32, bytes_after_slot: u32) -> u32 {
    unsafe { enet_crc32_slot_adjust(crc, old_slot, new_slot, bytes_after_slot) }
}

/// `crc32(&[a, b])` from `crc32(&[a])`, `crc32(&[b])` and `b.len()`: the merged digest of
/// shards checksummed on different GPUs (host arithmetic, no device work).
pub fn combine(crc_a: u32, crc_b: u32, len_b: u64) -> u32 {
    unsafe { enet_crc32_combine(crc_a, crc_b, len_b) }
}

#[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub struct CrcError {
    pub status: i32,
    pub hip_error: i32,
}

struct Ctx(*mut enet_crc_ctx);
// The C ABI serialises calls on one context with an internal lock.
unsafe impl Send for Ctx {}
unsafe impl Sync for Ctx {}
impl Drop for Ctx {
    fn drop(&mut self) {
        unsafe { enet_crc_ctx_destroy(self.0) }
    }
}

/// A device context; cheap to clone (shared).
#[derive(Clone)]
pub struct GpuCrc32 {
    ctx: Arc<Ctx>,
}

impl GpuCrc32 {
    pub fn new(device: i32) -> Result<Self, CrcError> {
        Self::with_devices(&[device])
    }

    /// A context over several GPUs (or lanes on one GPU: a device may repeat).  Host
    /// batches (`crc32_ragged_host`) are split into one byte-balanced shard per entry
    /// and checksummed on all of them at once.
    pub fn with_devices(devices: &[i32]) -> Result<Self, CrcError> {
        let mut p = core::ptr::null_mut();
        let st = unsafe { enet_crc_ctx_create_multi(devices.as_ptr(), devices.len() as u32, &mut p) };
        if st != ENET_CRC_OK {
            return Err(last_error(st));
        }
        Ok(Self { ctx: Arc::new(Ctx(p)) })
    }

    /// Every visible GPU of the node, one lane each.
    pub fn all_devices() -> Result<Self, CrcError> {
        let n = unsafe { enet_crc_device_count() };
        if n <= 0 {
            return Err(last_error(if n == 0 { -2 } else { n }));
        }
        let devs: Vec<i32> = (0..n).collect();
        Self::with_devices(&devs)
    }

    /// How `crc32` moves one datagram: `ENET_CRC_PERCALL_ZEROCOPY` (default: one launch
    /// per call, nothing resident), `ENET_CRC_PERCALL_COPY`, or `ENET_CRC_PERCALL_PERSISTENT`
    /// (opt-in: a server wave stays on the GPU while calls keep coming; a device-wide
    /// synchronize waits for it until `stop_server` or its 20-ms idle exit).
    /// None of them beats the CPU per datagram; batch instead.
    pub fn set_percall_mode(&self, mode: i32) -> Result<(), CrcError> {
        let st = unsafe { enet_crc_ctx_set_percall_mode(self.ctx.0, mode) };
        if st != ENET_CRC_OK {
            return Err(last_error(st));
        }
        Ok(())
    }

    /// Stop the persistent server wave now, if one runs.
    pub fn stop_server(&self) -> Result<(), CrcError> {
        let st = unsafe { enet_crc_ctx_stop_server(self.ctx.0) };
        if st != ENET_CRC_OK {
            return Err(last_error(st));
        }
        Ok(())
    }

    /// The device-side failure word of `device` (ABI 6): `Ok(0)` if no batch kernel gave
    /// up since the last clear, else the failure bits; check it (with `clear`) after the
    /// asynchronous device entries before trusting their outputs.  The host entries below
    /// return `ENET_CRC_E_DEVICE` (-5) instead.
    pub fn device_status(device: i32, clear: bool) -> Result<i32, CrcError> {
        let st = unsafe { enet_crc_device_status(device, clear as c_int) };
        if st < 0 {
            return Err(last_error(st));
        }
        Ok(st)
    }

    /// Same contract as `rusty_enet::crc32` (src/crc32.rs:39), but fallible.
    pub fn crc32(&self, in_buffers: &[&[u8]]) -> Result<u32, CrcError> {
        let iov: Vec<enet_crc_iov> =
            in_buffers.iter().map(|b| enet_crc_iov { data: b.as_ptr(), len: b.len() }).collect();
        let mut out = 0u32;
        let st = unsafe { enet_crc32_iov(self.ctx.0, iov.as_ptr(), iov.len(), &mut out) };
        if st != ENET_CRC_OK {
            return Err(CrcError { status: st, hip_error: unsafe { enet_crc_last_hip_error() } });
        }
        Ok(out)
    }

    /// The value for `HostSettings::checksum`.  The reference hook cannot
    /// fail, so a device error panics (fail loudly; there is no CPU fallback).
    pub fn checksum_fn(&self) -> Box<dyn Fn(&[&[u8]]) -> u32> {
        let me = self.clone();
        Box::new(move |bufs: &[&[u8]]| me.crc32(bufs).expect("enet_crc_amd: GPU checksum failed"))
    }

    /// Host-resident batch: one checksum per (offset, length) packet of `data`.
    pub fn crc32_ragged_host(&self, data: &[u8], offsets: &[u64], lengths: &[u32]) -> Result<Vec<u32>, CrcError> {
        assert_eq!(offsets.len(), lengths.len());
        for (o, l) in offsets.iter().zip(lengths) {
            assert!(*o as usize + *l as usize <= data.len(), "packet out of bounds");
        }
        let mut out = vec![0u32; offsets.len()];
        let st = unsafe {
            enet_crc32_ragged_host(self.ctx.0, data.as_ptr().cast(), offsets.as_ptr(), lengths.as_ptr(),
                                   offsets.len() as u64, out.as_mut_ptr())
        };
        if st != ENET_CRC_OK {
            return Err(CrcError { status: st, hip_error: unsafe { enet_crc_last_hip_error() } });
        }
        Ok(out)
    }
}

/// The `Compressor` of rusty_enet (src/compressor.rs:9-14) on the GPU: the range coder
/// of src/c/compress.rs, run by the `enet_range_*` entry points on a context that owns
/// the arenas.  Install with `HostSettings { compressor: Some(Box::new(gpu_rc)), .. }`.
pub struct GpuRangeCoder {
    ctx: Arc<Ctx>,
}

impl GpuRangeCoder {
    pub fn new(device: i32) -> Result<Self, CrcError> {
        Ok(Self { ctx: GpuCrc32::new(device)?.ctx })
    }

    /// Shares a checksum context (and so its device, lock and staging).
    pub fn from_crc(gpu: &GpuCrc32) -> Self {
        Self { ctx: gpu.ctx.clone() }
    }

    pub fn try_compress(&self, in_buffers: &[&[u8]], in_limit: usize, out: &mut [u8]) -> Result<usize, CrcError> {
        let iov: Vec<enet_crc_iov> =
            in_buffers.iter().map(|b| enet_crc_iov { data: b.as_ptr(), len: b.len() }).collect();
        let mut n = 0usize;
        let st = unsafe {
            enet_range_compress_iov(self.ctx.0, iov.as_ptr(), iov.len(), in_limit, out.as_mut_ptr(), out.len(), &mut n)
        };
        if st != ENET_CRC_OK {
            return Err(last_error(st));
        }
        Ok(n)
    }

    pub fn try_decompress(&self, in_data: &[u8], out: &mut [u8]) -> Result<usize, CrcError> {
        let mut n = 0usize;
        let st = unsafe {
            enet_range_decompress(self.ctx.0, in_data.as_ptr(), in_data.len(), out.as_mut_ptr(), out.len(), &mut n)
        };
        if st != ENET_CRC_OK {
            return Err(last_error(st));
        }
        Ok(n)
    }
}

/// `impl rusty_enet::Compressor for GpuRangeCoder` (enable the `rusty_enet` feature).
/// The trait has no error channel; a device failure panics (no CPU fallback).
#[cfg(feature = "rusty_enet")]
impl rusty_enet::Compressor for GpuRangeCoder {
    fn compress(&mut self, in_buffers: &[&[u8]], in_limit: usize, out: &mut [u8]) -> usize {
        self.try_compress(in_buffers, in_limit, out).expect("enet_crc_amd: GPU range coder failed")
    }

    fn decompress(&mut self, in_data: &[u8], out: &mut [u8]) -> usize {
        self.try_decompress(in_data, out).expect("enet_crc_amd: GPU range coder failed")
    }
}

#[cfg(test)]
mod test {
    // The reference's own known answers, src/crc32.rs:49-57.
    #[test]
    fn crc32() {
        let gpu = super::GpuCrc32::new(0).unwrap();
        assert_eq!(gpu.crc32(&[&[1, 2, 3, 4, 5, 6, 7, 8]]).unwrap(), 3314076223);
        assert_eq!(gpu.crc32(&[&[1, 2, 3, 4, 5, 6, 7, 8], &[8, 7, 6, 5, 4, 3, 2, 1]]).unwrap(), 1712484799);
    }

    #[test]
    fn range_round_trip() {
        let rc = super::GpuRangeCoder::new(0).unwrap();
        let data: Vec<u8> = (0..1000u32).map(|i| (i % 7) as u8).collect();
        let mut out = vec![0u8; 1000];
        let n = rc.try_compress(&[&data], data.len(), &mut out).unwrap();
        assert!(n > 0 && n < data.len());
        let mut back = vec![0u8; 4096];
        let m = rc.try_decompress(&out[..n], &mut back).unwrap();
        assert_eq!(&back[..m], &data[..]);
    }
}
