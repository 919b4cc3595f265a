from .netresdeep import NetResDeep, ResBlock  # noqa: F401
