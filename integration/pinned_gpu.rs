//! Download buffers in page-locked host memory.  New file for the reference crate:
//! `src/pinned_gpu.rs`.  Not compiled here (no cargo): checked textually by `tests/test_integration_cpu.py`.
//!
//! The reference downloads every chunk into an 8-byte aligned `Vec<u8>` (s3_client.rs:215-233,
//! chunk_downloader_http.rs:137-146: `maligned::align_first::<u8, A8>(content_length)` then
//! `extend_from_slice` of each body part) — pageable memory, so the engine's H2D of that chunk goes
//! through a staging copy in the HIP runtime.  `PinnedBuf` is the same buffer in the engine's
//! page-locked memory (`rdx_host_alloc`, page aligned: more than A8): the downloader fills it with the
//! same one copy per body part, and `rdx_execute*` DMAs it to HBM directly (the engine detects pinned
//! chunks; selects from pinned chunks into pinned results are pipelined).
//!
//! The downloaders fill it through `download_gpu.rs` (the patch to s3_client.rs:215-233 and
//! chunk_downloader_http.rs:137-146), with the GPU engine enabled;
//! and `app_gpu::operation_gpu` hands the resulting `Bytes` to the engine as a slice
//! (`operations_gpu::execute_slice`), never converting it to a `Vec`.

use std::os::raw::c_void;

use bytes::Bytes;

use crate::error::ActiveStorageError;
use crate::rdx_ffi::{rdx_host_alloc, rdx_host_free, status};

/// A page-locked download buffer of fixed capacity (the response's Content-Length).
pub struct PinnedBuf {
    ptr: *mut u8,
    len: usize,
    cap: usize,
}

// The buffer is plain host memory owned by this value; the engine's allocator is thread-safe.
unsafe impl Send for PinnedBuf {}
unsafe impl Sync for PinnedBuf {}

impl PinnedBuf {
    pub fn with_capacity(cap: usize) -> Result<Self, ActiveStorageError> {
        let mut p: *mut c_void = std::ptr::null_mut();
        let st = unsafe { rdx_host_alloc(crate::operations_gpu::context(), cap as u64, &mut p) };
        if st != status::OK || p.is_null() {
            return Err(ActiveStorageError::GpuEngine { status: st, error: "page-locked download buffer".into() });
        }
        Ok(PinnedBuf { ptr: p as *mut u8, len: 0, cap })
    }

    /// Append one part of the response body (the reference's `buf.extend_from_slice(&bytes)`); a body
    /// longer than its Content-Length is an error, as the aligned Vec could not have held it either
    /// without a reallocation the reference never expects.
    pub fn extend_from_slice(&mut self, part: &[u8]) -> Result<(), ActiveStorageError> {
        if self.len + part.len() > self.cap {
            return Err(ActiveStorageError::GpuEngine {
                status: status::E_BUFFER_TOO_SMALL,
                error: "response body longer than its content length".into(),
            });
        }
        unsafe { std::ptr::copy_nonoverlapping(part.as_ptr(), self.ptr.add(self.len), part.len()) };
        self.len += part.len();
        Ok(())
    }

    /// The downloaded chunk as `Bytes` owning this buffer (freed with rdx_host_free when the last clone
    /// drops — after the response and any chunk-cache entry holding it are gone).
    pub fn into_bytes(self) -> Bytes {
        Bytes::from_owner(self)
    }
}

impl AsRef<[u8]> for PinnedBuf {
    fn as_ref(&self) -> &[u8] {
        unsafe { std::slice::from_raw_parts(self.ptr, self.len) }
    }
}

impl Drop for PinnedBuf {
    fn drop(&mut self) {
        unsafe { rdx_host_free(crate::operations_gpu::context(), self.ptr as *mut c_void) }
    }
}
