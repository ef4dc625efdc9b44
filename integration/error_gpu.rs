//! The one addition the GPU plugins need in `src/error.rs` (reference error.rs:30-130 / 242-376): a
//! variant for failures that belong to the engine itself — HIP runtime errors, device faults, device or
//! page-locked memory exhaustion, no usable gfx950 device — reported as HTTP 500 (and logged, as every
//! 5xx is, error.rs:366-373).  Request-caused conditions keep the reference's variants (operations_gpu.rs
//! `check`), so clients see the same 4xx/5xx as from the CPU path.  Not compiled here (no cargo).

// 1. In `pub enum ActiveStorageError` (error.rs:30):
//
//     /// Error raised by the GPU engine (rdx_status of include/rdx.h)
//     #[error("GPU engine error {status}: {error}")]
//     GpuEngine { status: i32, error: String },
//
// 2. In `impl From<ActiveStorageError> for ErrorResponse` (error.rs:242), beside the other
//    internal-server-error arms:
//
//     ActiveStorageError::FromBytes { type_name: _ }
//     | ActiveStorageError::TryFromInt(_)
//     | ActiveStorageError::S3ByteStream(_)
//     | ActiveStorageError::SemaphoreAcquireError(_)
//     | ActiveStorageError::ChunkCacheError { error: _ }
//     | ActiveStorageError::GpuEngine { status: _, error: _ } => Self::internal_server_error(&error),
//
// 3. Test beside error.rs's own status tests (error.rs tests module):

#[cfg(test)]
mod gpu_engine_error_tests {
    use super::*;
    use axum::http::StatusCode;

    #[tokio::test]
    async fn gpu_engine_error_is_500() {
        let error = ActiveStorageError::GpuEngine { status: 9, error: "device error".into() };
        let message = "GPU engine error 9: device error";
        let caused_by = None;
        test_active_storage_error(error, StatusCode::INTERNAL_SERVER_ERROR, message, caused_by).await;
    }
}
