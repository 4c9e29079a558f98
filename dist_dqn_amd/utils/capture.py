"""Guard for HIP graph captures on the training thread.

A capture forbids most runtime calls on the capturing thread. Two host-side sources of such
calls can fire mid-capture without the capturing code issuing them: a Python garbage-collection
pass (a destructor of a snapshot buffer or an event) and the asynchronous checkpoint writer
(D2H copies, event waits, snapshot frees on its own thread). ``quiet_capture()`` joins the
writers and keeps the collector off for the duration of the capture.
"""
import contextlib
import gc


@contextlib.contextmanager
def quiet_capture():
    from ..checkpoint import quiesce_writers
    quiesce_writers()
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()
