"""MI355X-native Sequential Routing Framework (SRF) hot path.

Host side mirrors tfsr's interface (SequenceRouter, trainer_sr step functions,
ParseOption flags); compute runs in the HIP library ``libsrf.so`` behind the C
ABI declared in ``include/srf.h``.
"""
__version__ = '0.1.0'
