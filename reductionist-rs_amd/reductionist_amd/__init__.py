"""MI355X (gfx950) chunk filter+reduce engine — drop-in for reductionist-rs's synchronous request
path (src/app.rs:163-183).  Host mirror of the reference's Operation plugin surface over the C ABI
in include/rdx.h; all data-path work runs in hand-written HIP kernels (csrc/)."""
from . import _abi
from .engine import Engine, Workspace
from .errors import ActiveStorageError
from .models import RequestData, Response
from .operations import OPERATIONS, Count, Max, Min, Select, Sum, operation

__all__ = ["Engine", "Workspace", "ActiveStorageError", "RequestData", "Response", "OPERATIONS", "Count", "Max",
           "Min", "Select", "Sum", "operation", "_abi"]
