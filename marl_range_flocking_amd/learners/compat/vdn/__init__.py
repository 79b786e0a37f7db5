"""vdn package shim (learners/vdn/)."""
