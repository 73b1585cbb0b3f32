//! The surface helyim-ec uses, on libhec: `ReedSolomon::{new, encode, verify,
//! reconstruct, reconstruct_data}` (reed_solomon_erasure 6.0.0, used at
//! /root/reference/helyim-ec/src/encoder.rs:191,208-209,249-250,288 and
//! helyim-store/src/erasure_coding/mod.rs:411-412,426), the batched degraded
//! read, and `write_ec_files` / `rebuild_ec_files`
//! (helyim-ec/src/encoder.rs:39-50).
//!
//! The swap in helyim: `use helyim_ec_hip::ReedSolomon`
//! for `use reed_solomon_erasure::{ReedSolomon, galois_8::Field}` at each call
//! site, and `#[from] helyim_ec_hip::Error` for `#[from]
//! reed_solomon_erasure::Error` at helyim-ec/src/errors.rs:27,59. `Error` has
//! upstream's 13 variants in upstream's order and Display text, plus
//! `Device` for libhec's own failures (no GPU, HIP errors), which reaches gRPC
//! as `Status::internal` through helyim's existing `From<..> for Status`
//! impls (errors.rs:37-41, 68-72). `EcShardError` has helyim's exact shape
//! (errors.rs:54-66), payloads included.

use std::ffi::{CStr, CString};
use std::fmt;
use std::io;
use std::os::raw::c_int;

use hec_sys as sys;

/// reed_solomon_erasure::Error, declaration order (codes 1..=13), plus
/// libhec's device / argument failures (codes >= 64).
#[derive(Clone, Debug, PartialEq, Eq)]
pub enum Error {
    TooFewShards,
    TooManyShards,
    TooFewDataShards,
    TooManyDataShards,
    TooFewParityShards,
    TooManyParityShards,
    TooFewBufferShards,
    TooManyBufferShards,
    IncorrectShardSize,
    TooFewShardsPresent,
    EmptyShard,
    InvalidShardFlags,
    InvalidIndex,
    /// libhec device / argument failure: (status code, hec_last_error_detail).
    /// No upstream variant; helyim maps it to `Status::internal` like the rest.
    Device(i32, String),
}

impl fmt::Display for Error {
    /// Upstream 6.0.0's Display text for the 13 variants (the same strings
    /// `hec_strerror` returns for codes 1..=13).
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        use Error::*;
        let text = match self {
            TooFewShards => "The number of provided shards is smaller than the one in codec",
            TooManyShards => "The number of provided shards is greater than the one in codec",
            TooFewDataShards => "The number of provided data shards is smaller than the one in codec",
            TooManyDataShards => "The number of provided data shards is greater than the one in codec",
            TooFewParityShards => "The number of provided parity shards is smaller than the one in codec",
            TooManyParityShards => "The number of provided parity shards is greater than the one in codec",
            TooFewBufferShards => "The number of provided buffer shards is smaller than the number of parity shards in codec",
            TooManyBufferShards => "The number of provided buffer shards is greater than the number of parity shards in codec",
            IncorrectShardSize => "At least one of the provided shards is not of the correct size",
            TooFewShardsPresent => "The number of shards present is smaller than number of parity shards, cannot reconstruct missing shards",
            EmptyShard => "The first shard provided is of zero length",
            InvalidShardFlags => "The number of flags does not match the total number of shards",
            InvalidIndex => "The data shard index provided is greater or equal to the number of data shards in codec",
            Device(code, detail) => {
                let what = unsafe { CStr::from_ptr(sys::hec_strerror(*code)) }.to_string_lossy();
                return if detail.is_empty() {
                    write!(f, "libhec error {code}: {what}")
                } else {
                    write!(f, "libhec error {code}: {what} ({detail})")
                };
            }
        };
        f.write_str(text)
    }
}

impl std::error::Error for Error {}

/// The variant of a status code (codes 1..=13 upstream's, anything else
/// `Device` with this thread's failure detail).
pub fn to_err(code: c_int) -> Error {
    use Error::*;
    match code {
        1 => TooFewShards,
        2 => TooManyShards,
        3 => TooFewDataShards,
        4 => TooManyDataShards,
        5 => TooFewParityShards,
        6 => TooManyParityShards,
        7 => TooFewBufferShards,
        8 => TooManyBufferShards,
        9 => IncorrectShardSize,
        10 => TooFewShardsPresent,
        11 => EmptyShard,
        12 => InvalidShardFlags,
        13 => InvalidIndex,
        c => Device(c, last_error_detail()),
    }
}

fn check(code: c_int) -> Result<(), Error> {
    if code == sys::HEC_OK { Ok(()) } else { Err(to_err(code)) }
}

/// The text libhec gives for the last failure on this thread.
pub fn last_error_detail() -> String {
    unsafe { CStr::from_ptr(sys::hec_last_error_detail()) }.to_string_lossy().into_owned()
}

/// (a, b, errno) of the last failure on this thread (`hec_last_error_values`):
/// the two usizes of the size variants, the OS error behind an Io.
pub fn last_error_values() -> (u64, u64, i32) {
    let (mut a, mut b, mut e) = (0u64, 0u64, 0 as c_int);
    unsafe { sys::hec_last_error_values(&mut a, &mut b, &mut e) };
    (a, b, e)
}

pub struct ReedSolomon(*mut sys::hec_rs_t);
unsafe impl Send for ReedSolomon {}
unsafe impl Sync for ReedSolomon {} // immutable after new; libhec's device state is mutex-guarded

impl ReedSolomon {
    pub fn new(data_shards: usize, parity_shards: usize) -> Result<Self, Error> {
        let mut h = std::ptr::null_mut();
        check(unsafe { sys::hec_rs_new(data_shards, parity_shards, &mut h) })?;
        Ok(Self(h))
    }

    pub fn raw(&self) -> *const sys::hec_rs_t {
        self.0
    }

    pub fn data_shard_count(&self) -> usize {
        unsafe { sys::hec_rs_data_shard_count(self.0) }
    }

    pub fn parity_shard_count(&self) -> usize {
        unsafe { sys::hec_rs_parity_shard_count(self.0) }
    }

    pub fn total_shard_count(&self) -> usize {
        unsafe { sys::hec_rs_total_shard_count(self.0) }
    }

    /// Parity of shards[0..data] into shards[data..total], in place. Upstream's
    /// signature (reed_solomon_erasure 6.0.0 `ReedSolomon::encode<T, U>(&self,
    /// shards: T)`), so `reed_solomon.encode(bufs.as_mut())` at
    /// helyim-ec/src/encoder.rs:191 binds unchanged.
    pub fn encode<T, U>(&self, mut shards: T) -> Result<(), Error>
    where
        T: AsRef<[U]> + AsMut<[U]>,
        U: AsRef<[u8]> + AsMut<[u8]>,
    {
        let slices = shards.as_mut();
        let lens: Vec<usize> = slices.iter().map(|s| s.as_ref().len()).collect();
        let ptrs: Vec<*mut u8> = slices.iter_mut().map(|s| s.as_mut().as_mut_ptr()).collect();
        check(unsafe { sys::hec_rs_encode(self.0, ptrs.as_ptr(), lens.as_ptr(), ptrs.len()) })
    }

    pub fn verify<T: AsRef<[u8]>>(&self, shards: &[T]) -> Result<bool, Error> {
        let lens: Vec<usize> = shards.iter().map(|s| s.as_ref().len()).collect();
        let ptrs: Vec<*const u8> = shards.iter().map(|s| s.as_ref().as_ptr()).collect();
        let mut ok = 0;
        check(unsafe { sys::hec_rs_verify(self.0, ptrs.as_ptr(), lens.as_ptr(), ptrs.len(), &mut ok) })?;
        Ok(ok == 1)
    }

    /// Upstream semantics and signature (`reconstruct<T: ReconstructShard<F>>(&self,
    /// shards: &mut [T])`): `reconstruct(&mut bufs)` at encoder.rs:288 and
    /// erasure_coding/mod.rs:426 binds unchanged. Missing `None` slots are
    /// allocated `vec![0; len]` and filled; on error the slots are left as
    /// they were.
    pub fn reconstruct<T: ReconstructShard>(&self, shards: &mut [T]) -> Result<(), Error> {
        self.reconstruct_impl(shards, false)
    }

    /// As `reconstruct`, but missing parity slots stay absent.
    pub fn reconstruct_data<T: ReconstructShard>(&self, shards: &mut [T]) -> Result<(), Error> {
        self.reconstruct_impl(shards, true)
    }

    fn reconstruct_impl<T: ReconstructShard>(&self, shards: &mut [T], data_only: bool) -> Result<(), Error> {
        let present: Vec<u8> = shards.iter().map(|s| s.len().is_some() as u8).collect();
        let lens: Vec<usize> = shards.iter().map(|s| s.len().unwrap_or(0)).collect();
        let len = lens.iter().copied().find(|&l| l > 0).unwrap_or(0);
        let k = self.data_shard_count();
        let mut ptrs: Vec<*mut u8> = Vec::with_capacity(shards.len());
        let mut init_err = None;
        for s in shards.iter_mut() {
            match s.get_or_initialize(len) {
                Ok(b) => ptrs.push(b.as_mut_ptr()),
                Err(e) => {
                    init_err = Some(e);
                    break;
                }
            }
        }
        if let Some(e) = init_err {
            for (t, &p) in shards.iter_mut().zip(&present) {
                if p == 0 {
                    t.reset(); // nothing written: absent slots stay absent
                }
            }
            return Err(e);
        }
        let rc = unsafe {
            if data_only {
                sys::hec_rs_reconstruct_data(self.0, ptrs.as_ptr(), lens.as_ptr(), present.as_ptr(), ptrs.len())
            } else {
                sys::hec_rs_reconstruct(self.0, ptrs.as_ptr(), lens.as_ptr(), present.as_ptr(), ptrs.len())
            }
        };
        for (i, (s, &p)) in shards.iter_mut().zip(&present).enumerate() {
            if p == 0 && (rc != 0 || (data_only && i >= k)) {
                s.reset(); // untouched on error; reconstruct_data leaves parity absent
            }
        }
        check(rc)
    }

    /// Many independent stripes (e.g. all lost intervals of a needle read,
    /// erasure_coding/mod.rs:403-491) in ONE GPU round trip. Stripe j is
    /// `stripes[j]`, each with upstream `reconstruct` semantics. On error
    /// nothing is written and the error names the first failing stripe.
    pub fn reconstruct_batch(&self, stripes: &mut [Vec<Option<Vec<u8>>>]) -> Result<(), (Error, usize)> {
        let n = self.total_shard_count();
        // hec_rs_reconstruct_batch reads exactly n entries per stripe: a stripe
        // of another length would shift every later stripe's shards (and read
        // past the arrays), so it is refused first, as upstream's per-call
        // check_piece_count! does
        for (j, st) in stripes.iter().enumerate() {
            if st.len() < n {
                return Err((Error::TooFewShards, j));
            }
            if st.len() > n {
                return Err((Error::TooManyShards, j));
            }
        }
        let mut ptrs = Vec::with_capacity(stripes.len() * n);
        let mut lens = Vec::with_capacity(stripes.len() * n);
        let mut present = Vec::with_capacity(stripes.len() * n);
        for st in stripes.iter_mut() {
            let len = st.iter().flatten().map(|b| b.len()).next().unwrap_or(0);
            for b in st.iter_mut() {
                present.push(b.is_some() as u8);
                lens.push(b.as_ref().map_or(0, |v| v.len()));
                ptrs.push(b.get_or_insert_with(|| vec![0u8; len]).as_mut_ptr());
            }
        }
        let mut bad = 0usize;
        let rc = unsafe {
            sys::hec_rs_reconstruct_batch(self.0, ptrs.as_ptr(), lens.as_ptr(), present.as_ptr(), stripes.len(), 0,
                                          &mut bad)
        };
        if rc != 0 {
            let mut it = present.iter();
            for st in stripes.iter_mut() {
                for b in st.iter_mut() {
                    if *it.next().unwrap() == 0 {
                        *b = None;
                    }
                }
            }
            return Err((to_err(rc), bad));
        }
        Ok(())
    }
}

/// The shard slots `reconstruct` accepts (upstream `ReconstructShard<F>` for
/// `galois_8::Field`): `Option<Vec<u8>>` (absent = `None`, allocated on
/// reconstruct) and `(buffer, present)` pairs whose buffer is caller storage.
pub trait ReconstructShard {
    /// Length of a present shard; `None` when the slot is absent.
    fn len(&self) -> Option<usize>;
    /// The slot's bytes, allocating `len` zero bytes for an absent
    /// `Option` slot; an absent pair slot whose buffer is not `len` long is
    /// `IncorrectShardSize`.
    fn get_or_initialize(&mut self, len: usize) -> Result<&mut [u8], Error>;
    /// Back to absent after a failed or data-only reconstruct.
    fn reset(&mut self);
}

impl ReconstructShard for Option<Vec<u8>> {
    fn len(&self) -> Option<usize> {
        self.as_ref().map(|v| v.len())
    }
    fn get_or_initialize(&mut self, len: usize) -> Result<&mut [u8], Error> {
        Ok(self.get_or_insert_with(|| vec![0u8; len]).as_mut_slice())
    }
    fn reset(&mut self) {
        *self = None;
    }
}

impl<T: AsRef<[u8]> + AsMut<[u8]>> ReconstructShard for (T, bool) {
    fn len(&self) -> Option<usize> {
        if self.1 { Some(self.0.as_ref().len()) } else { None }
    }
    fn get_or_initialize(&mut self, len: usize) -> Result<&mut [u8], Error> {
        if !self.1 && self.0.as_ref().len() != len {
            return Err(Error::IncorrectShardSize);
        }
        self.1 = true; // filled by the reconstruct (reset() undoes it on failure)
        Ok(self.0.as_mut())
    }
    fn reset(&mut self) {
        self.1 = false;
    }
}

impl ReedSolomon {
    /// Stripe count of a packed `[S][total][L]` host batch, or the upstream
    /// error a wrong size maps to.
    fn packed_stripes(&self, bytes: usize, shard_len: usize) -> Result<u32, Error> {
        let stripe = self.total_shard_count().checked_mul(shard_len).ok_or(Error::IncorrectShardSize)?;
        if shard_len == 0 {
            return Err(Error::EmptyShard);
        }
        if bytes % stripe != 0 {
            return Err(Error::IncorrectShardSize);
        }
        u32::try_from(bytes / stripe).map_err(|_| Error::TooManyShards)
    }

    /// One packed host batch `[S][total][L]` (parity written in place into
    /// shards data..total of every stripe), split into contiguous stripe
    /// ranges over `devices` (`hec_host_encode_batch_multi`; a device may
    /// repeat). Pinned memory (`hec_host_alloc`) is coded zero-copy.
    pub fn encode_batch_multi(&self, devices: &[i32], stripes: &mut [u8], shard_len: usize) -> Result<(), Error> {
        let s = self.packed_stripes(stripes.len(), shard_len)?;
        let (n, k, l) = (self.total_shard_count() as u64, self.data_shard_count() as u64, shard_len as u64);
        let base = stripes.as_mut_ptr();
        check(unsafe {
            sys::hec_host_encode_batch_multi(self.0, devices.as_ptr(), devices.len(), base, n * l, l,
                                             base.wrapping_add((k * l) as usize), n * l, l, l, s)
        })
    }

    /// In-place reconstruct of a packed `[S][total][L]` host batch over
    /// `devices` (`hec_host_reconstruct_batch_multi`); `present_masks[s]` bit i
    /// = shard i of stripe s present. Returns the stripes skipped for too few
    /// present shards.
    pub fn reconstruct_batch_multi(&self, devices: &[i32], stripes: &mut [u8], shard_len: usize,
                                   present_masks: &[u32]) -> Result<u32, Error> {
        let s = self.packed_stripes(stripes.len(), shard_len)?;
        if present_masks.len() != s as usize {
            return Err(Error::InvalidShardFlags);
        }
        let (n, l) = (self.total_shard_count() as u64, shard_len as u64);
        let mut bad = 0u32;
        check(unsafe {
            sys::hec_host_reconstruct_batch_multi(self.0, devices.as_ptr(), devices.len(), stripes.as_mut_ptr(),
                                                  n * l, l, l, s, present_masks.as_ptr(), &mut bad)
        })?;
        Ok(bad)
    }
}

impl Drop for ReedSolomon {
    fn drop(&mut self) {
        unsafe { sys::hec_rs_free(self.0) }
    }
}

/// helyim_ec::EcShardError with helyim's exact variants and payloads
/// (helyim-ec/src/errors.rs:54-66). libhec's device failures arrive as
/// `ErasureCoding(Error::Device(..))`, so no variant is added.
#[derive(Debug)]
pub enum EcShardError {
    Io(io::Error),
    ErasureCoding(Error),
    Underflow(usize, usize),
    UnexpectedEcShardSize(usize, usize),
    UnexpectedBlockSize(usize, usize),
}

impl fmt::Display for EcShardError {
    /// helyim's thiserror formats (errors.rs:56-65), Underflow's `{0}` twice included.
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        match self {
            EcShardError::Io(e) => write!(f, "Io error: {e}"),
            EcShardError::ErasureCoding(e) => write!(f, "Erasure coding error: {e}"),
            EcShardError::Underflow(a, _) => write!(f, "Only {a} shards found but {a} required"),
            EcShardError::UnexpectedEcShardSize(a, b) => write!(f, "ec shard size expected {a} but actually is {b}"),
            EcShardError::UnexpectedBlockSize(a, b) => write!(f, "unexpected block size {a}, buffer size {b}"),
        }
    }
}

impl std::error::Error for EcShardError {
    fn source(&self) -> Option<&(dyn std::error::Error + 'static)> {
        match self {
            EcShardError::Io(e) => Some(e),
            EcShardError::ErasureCoding(e) => Some(e),
            _ => None,
        }
    }
}

impl From<io::Error> for EcShardError {
    fn from(e: io::Error) -> Self {
        EcShardError::Io(e)
    }
}

impl From<Error> for EcShardError {
    fn from(e: Error) -> Self {
        EcShardError::ErasureCoding(e)
    }
}

/// The EcShardError of a file-layer status, payload from
/// `hec_last_error_values` (codes 32..=35; RS and device codes wrap as
/// `ErasureCoding`, like errors.rs:58-59).
fn file_err(code: c_int) -> EcShardError {
    let (a, b, errno) = last_error_values();
    match code {
        sys::HEC_ERR_IO if errno != 0 => EcShardError::Io(io::Error::from_raw_os_error(errno)),
        sys::HEC_ERR_IO => EcShardError::Io(io::Error::new(io::ErrorKind::Other, last_error_detail())),
        sys::HEC_ERR_UNDERFLOW => EcShardError::Underflow(a as usize, b as usize),
        sys::HEC_ERR_UNEXPECTED_EC_SHARD_SIZE => EcShardError::UnexpectedEcShardSize(a as usize, b as usize),
        sys::HEC_ERR_UNEXPECTED_BLOCK_SIZE => EcShardError::UnexpectedBlockSize(a as usize, b as usize),
        c => EcShardError::ErasureCoding(to_err(c)),
    }
}

fn cstr(s: &str) -> Result<CString, EcShardError> {
    CString::new(s).map_err(|e| EcShardError::Io(io::Error::new(io::ErrorKind::InvalidInput, e)))
}

/// helyim_ec::write_ec_files (encoder.rs:39-46): base.dat -> base.ec00..ec13.
pub fn write_ec_files(base_filename: &str) -> Result<(), EcShardError> {
    let c = cstr(base_filename)?;
    match unsafe { sys::hec_write_ec_files(c.as_ptr()) } {
        0 => Ok(()),
        code => Err(file_err(code)),
    }
}

/// helyim_ec::rebuild_ec_files (encoder.rs:48-50): the rebuilt shard ids.
pub fn rebuild_ec_files(base_filename: &str) -> Result<Vec<u32>, EcShardError> {
    let c = cstr(base_filename)?;
    let mut ids = [0u32; 14];
    let mut n = 0usize;
    match unsafe { sys::hec_rebuild_ec_files(c.as_ptr(), ids.as_mut_ptr(), &mut n) } {
        0 => Ok(ids[..n].to_vec()),
        code => Err(file_err(code)),
    }
}

/// Pinned host memory for the host-batch calls, freed on drop
/// (`hec_host_alloc` / `hec_host_alloc_multi` + `hec_host_free`). Pinned
/// batches are coded zero-copy.
pub struct PinnedBuffer {
    ptr: *mut u8,
    len: usize,
}
unsafe impl Send for PinnedBuffer {}
unsafe impl Sync for PinnedBuffer {}

impl PinnedBuffer {
    /// `bytes` on the current device's NUMA node.
    pub fn new(bytes: usize) -> Result<Self, Error> {
        let mut p = std::ptr::null_mut();
        check(unsafe { sys::hec_host_alloc(bytes, &mut p) })?;
        Ok(Self { ptr: p as *mut u8, len: bytes })
    }

    /// One packed `[S][total][L]` batch for `encode_batch_multi` /
    /// `reconstruct_batch_multi` over `devices`: each device's stripe range
    /// has its pages on that device's NUMA node (`hec_host_alloc_multi`).
    pub fn for_devices(devices: &[i32], stripe_stride: u64, n_stripes: u32) -> Result<Self, Error> {
        let mut p = std::ptr::null_mut();
        check(unsafe { sys::hec_host_alloc_multi(devices.as_ptr(), devices.len(), stripe_stride, n_stripes, &mut p) })?;
        Ok(Self { ptr: p as *mut u8, len: (stripe_stride * n_stripes as u64) as usize })
    }
}

impl std::ops::Deref for PinnedBuffer {
    type Target = [u8];
    fn deref(&self) -> &[u8] {
        unsafe { std::slice::from_raw_parts(self.ptr, self.len) }
    }
}

impl std::ops::DerefMut for PinnedBuffer {
    fn deref_mut(&mut self) -> &mut [u8] {
        unsafe { std::slice::from_raw_parts_mut(self.ptr, self.len) }
    }
}

impl Drop for PinnedBuffer {
    fn drop(&mut self) {
        unsafe { sys::hec_host_free(self.ptr as *mut std::os::raw::c_void) };
    }
}

/// Multi-GPU servers: whole volumes per GPU, chosen on the
/// calling thread before the file-layer call.
pub fn select_device_for_volume(volume_id: u32) -> Result<i32, Error> {
    let mut n = 0;
    check(unsafe { sys::hec_device_count(&mut n) })?;
    let d = (volume_id % n.max(1) as u32) as i32;
    check(unsafe { sys::hec_set_device(d) })?;
    Ok(d)
}
