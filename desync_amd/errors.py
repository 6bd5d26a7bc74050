"""Errors of the chunking path (errors.go:56-58)."""


class Interrupted(Exception):
    """Returned when a chunking operation is cancelled (make.go:201-203)."""

    def __str__(self):
        return "interrupted"
