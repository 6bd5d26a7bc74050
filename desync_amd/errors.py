"""Errors of the chunking path (errors.go:56-58)."""


class Interrupted(Exception):
    """Returned when a chunking operation is cancelled (make.go:201-203)."""

    def __str__(self):
        return "interrupted"


class ChunkInvalid(Exception):
    """errors.go:23-43: a chunk's data does not hash to its ID (``Sum`` set),
    or its storage data could not be converted (``Err`` set)."""

    def __init__(self, ID: bytes, Sum: bytes = None, Err: BaseException = None):
        super().__init__(ID, Sum, Err)
        self.ID, self.Sum, self.Err = bytes(ID), (bytes(Sum) if Sum is not None else None), Err

    def __str__(self):
        if self.Err is not None:
            return f"invalid chunk {self.ID.hex()}: {self.Err}"
        return f"chunk id {self.ID.hex()} does not match its hash {(self.Sum or b'').hex()}"
