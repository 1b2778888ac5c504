"""gochugaru_amd — MI355X-native batched permission checks behind gochugaru's check API.

Package layout (only what the north-star path needs):

* ``rel``          — mirror of gochugaru's ``rel`` package (check item / ingest record)
* ``consistency``  — mirror of gochugaru's ``consistency`` package
* ``client``       — mirror of ``client.Client``'s check family, answered by the GPU engine
* ``engine``       — ctypes binding of ``libgck.so`` (C ABI: ``include/gck.h``)
* ``csrc/``        — C++ host data plane + HIP (gfx950) kernels behind that ABI
"""
from . import consistency, rel  # noqa: F401

__all__ = ["rel", "consistency", "client", "engine"]
