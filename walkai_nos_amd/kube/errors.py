"""API errors mirroring ``k8s.io/apimachinery/pkg/api/errors``."""


class APIError(Exception):
    code = 500


class NotFound(APIError):
    code = 404


class AlreadyExists(APIError):
    code = 409


class Conflict(APIError):
    code = 409


class Forbidden(APIError):
    code = 403


def is_not_found(e: BaseException) -> bool:
    return isinstance(e, NotFound)


def ignore_not_found(e: BaseException) -> None:
    if not isinstance(e, NotFound):
        raise e
