"""mtaz: MI355X-native AlphaZero self-play for MinitChess (drop-in for the
reference's exp/agent.py + exp/environment.py + exp/policy.py hot path).

Layout:
  csrc/            HIP kernels (gfx950) + C ABI (include/mtaz.h) -> libmtaz.so
  _lib.py          ctypes binding (fails loudly when the HIP library is missing)
  engine.py        batched self-play engine (one per GPU)
  environment.py   drop-in exp/environment.py (rules in libmtaz)
  network.py       drop-in exp/policy.py Network (weights container)
  agent.py, policy.py, callbacks.py, erlyx_compat.py, puppet.py
                   the reference's plugin surface and the app/puppet entry point
"""
__all__ = ['build', 'Engine']


def __getattr__(name):
    if name == 'Engine':
        from .engine import Engine
        return Engine
    if name == 'build':
        from .build import build
        return build
    raise AttributeError(name)
