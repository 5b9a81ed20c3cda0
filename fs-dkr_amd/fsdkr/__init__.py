"""fsdkr — MI355X-native batch verifier for FS-DKR's key-refresh hot path.

Host-side mirror of the reference operator API (Leo-Li009/fs-dkr,
src/refresh_message.rs, src/zk_pdl_with_slack.rs, src/range_proofs.rs,
src/ring_pedersen_proof.rs) over the C ABI in include/fsdkr/fsdkr.h."""
from ._native import Context, FsdkrError, lib  # noqa: F401
