"""Inert space classes (the reference only constructs them)."""


class _Space:
    def __init__(self, *args, **kwargs):
        self.args = args
        self.kwargs = kwargs


class Discrete(_Space):
    pass


class MultiDiscrete(_Space):
    pass


class Box(_Space):
    pass


class MultiBinary(_Space):
    pass


class Dict(_Space):
    pass
