from .arena import ParamArena, arena_of  # noqa: F401
