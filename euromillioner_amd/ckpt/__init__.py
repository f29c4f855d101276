"""ckpt subpackage."""
