"""Stand-in for ``pettingzoo.ParallelEnv`` (TEST INFRASTRUCTURE): only ``unwrapped``."""


class ParallelEnv:
    @property
    def unwrapped(self):
        return self
