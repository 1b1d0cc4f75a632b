"""GPU errors (reference ``pkg/gpu/errors.go:24-99``)."""
from __future__ import annotations

from typing import Iterable, List, Optional


class GpuError(Exception):
    NOT_FOUND = "not_found"
    GENERIC = "generic"
    PERMISSION = "permission"
    BUSY = "busy"

    def __init__(self, message: str, code: str = GENERIC):
        super().__init__(message)
        self.code = code

    def is_not_found(self) -> bool:
        return self.code == self.NOT_FOUND


def not_found(msg: str = "not found") -> GpuError:
    return GpuError(msg, GpuError.NOT_FOUND)


def generic(msg: str) -> GpuError:
    return GpuError(msg, GpuError.GENERIC)


def is_not_found(e: Optional[BaseException]) -> bool:
    return isinstance(e, GpuError) and e.is_not_found()


def ignore_not_found(e: Optional[BaseException]) -> Optional[BaseException]:
    return None if is_not_found(e) else e


class ErrorList(GpuError):
    def __init__(self, errors: Iterable[BaseException]):
        self.errors: List[BaseException] = list(errors)
        super().__init__("; ".join(str(e) for e in self.errors))
