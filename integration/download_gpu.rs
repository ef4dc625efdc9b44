//! The downloaders' change for the GPU engine: chunks land in page-locked host
//! memory, so the engine's H2D copy of a chunk is one DMA at full PCIe rate instead of a staging copy in the
//! HIP runtime.  New file for the reference crate: `src/download_gpu.rs` (declared in
//! `lib.rs` next to `pinned_gpu`).  Not compiled here (no cargo): checked textually by
//! `tests/test_integration_cpu.py`.
//!
//! Patch, in the form of `app_gpu.rs` (the lines each call replaces; everything before them — the request,
//! the Content-Length check, the resource manager's memory permits — stays as it is):
//!
//! * `src/s3_client.rs:215-233` (`S3Client::download_object`, from the aligned `Vec` to `Ok(buf.into())`):
//!
//!   ```ignore
//!   if crate::download_gpu::enabled() {
//!       return crate::download_gpu::s3_body(&mut response.body, content_length).await;
//!   }
//!   // ... the reference's maligned::align_first / extend_from_slice / Ok(buf.into()) otherwise
//!   ```
//!
//! * `src/chunk_downloader_http.rs:137-146` (the HTTP downloader, same span):
//!
//!   ```ignore
//!   if crate::download_gpu::enabled() {
//!       return crate::download_gpu::http_body(response, content_length).await;
//!   }
//!   ```
//!
//! `enabled()` is true once `app_gpu::init_gpu` has created the engine (`--use-gpu`); without it the
//! reference's code path runs unchanged.  Both bodies are copied once per body part into the
//! `PinnedBuf`, as the reference copies them once into its 8-byte aligned `Vec` (a page is a stronger
//! alignment than A8); a body longer than its Content-Length is an error here, where the reference's `Vec`
//! would have grown — the header is what the memory permits were taken for.

use bytes::Bytes;
use tokio_stream::StreamExt;
use tracing::Instrument;

use crate::error::ActiveStorageError;
use crate::pinned_gpu::PinnedBuf;

/// Whether downloads go to page-locked buffers: the GPU engine exists (created by `app_gpu::init_gpu`).
pub fn enabled() -> bool {
    crate::operations_gpu::initialized()
}

/// S3: the streaming body of a GetObject response into a page-locked buffer of `content_length` bytes.
pub async fn s3_body(
    body: &mut aws_sdk_s3::primitives::ByteStream,
    content_length: usize,
) -> Result<Bytes, ActiveStorageError> {
    let mut buf = PinnedBuf::with_capacity(content_length)?;
    while let Some(part) = body.try_next().instrument(tracing::Span::current()).await? {
        buf.extend_from_slice(&part)?;
    }
    Ok(buf.into_bytes())
}

/// HTTP: the response body, part by part as it arrives (no intermediate whole-body `Bytes`), into a
/// page-locked buffer of `content_length` bytes.
pub async fn http_body(mut response: reqwest::Response, content_length: usize) -> Result<Bytes, ActiveStorageError> {
    let mut buf = PinnedBuf::with_capacity(content_length)?;
    while let Some(part) = response.chunk().await? {
        buf.extend_from_slice(&part)?;
    }
    Ok(buf.into_bytes())
}
