"""Weight gradients on a side stream.

A layer's weight gradient (an in-place accumulation into the flat-buffer ``.grad``) and its input gradient are
independent: launching the weight gradient on a side stream that first waits for the compute stream lets the two
GEMMs / convolutions run side by side and fill each other's tails and tile rounds (GPT-2 step +1.7 %,
``profiles/r6_wgrad_side_stream_ab.jsonl``). The compute stream waits for the side stream at the end of every backward
pass (an autograd-engine callback queued by the first side launch of the pass, so a plain ``loss.backward()`` followed
by an optimizer step is safe) and wherever the engine synchronises or steps a stage's gradients
(``join_side_streams``). Never used while a HIP graph is being captured. ``SDML_WGRAD_STREAM=0`` keeps every launch on
the compute stream.

Operand lifetime: by default (``SDML_SIDE_HOLD=1``) the operands of every side launch are held here until the join, and
released only after the compute stream has waited for the side stream, so the caching allocator reuses their blocks in
compute-stream order - the same blocks every step. ``SDML_SIDE_HOLD=0`` uses ``record_stream`` instead: a freed block
then waits for the side stream's progress at reuse time, and the allocator's choices vary with timing.
"""
from __future__ import annotations

import os

import torch

WGRAD_STREAM = os.environ.get("SDML_WGRAD_STREAM", "1") == "1"
# the convolutions' weight gradients (ResNet). With record_stream: +3.7 % on one run and -12 / -26 % on two others of
# the same A/B (profiles/r6_side_stream_ab.jsonl). With the operands held to the join and the weight gradient enqueued
# after the input gradient (CONV_WGRAD_AFTER): 121.9-122.3 K samples/s in 3 of 4 runs, 113.7 K in one, against
# 113.5-117.0 K on the compute stream (profiles/r6_conv_side_order_ab.jsonl): on by default
CONV_WGRAD_STREAM = os.environ.get("SDML_CONV_WGRAD_STREAM", "1") == "1"
HOLD = os.environ.get("SDML_SIDE_HOLD", "1") == "1"
# conv weight gradients: enqueued after the input gradient (waiting on an event recorded before it), so the input
# gradient's workgroups are dispatched first and the weight gradient fills the CUs its last round leaves free
CONV_WGRAD_AFTER = os.environ.get("SDML_CONV_WGRAD_AFTER", "1") == "1"
_SIDE = {}
_PENDING = []
_HELD = []


def _side_stream(dev):
    s = _SIDE.get(dev.index)
    if s is None:
        s = _SIDE[dev.index] = torch.cuda.Stream(device=dev)
    return s


def join_side_streams():
    """The compute stream waits for every side-stream launch issued since the last join."""
    while _PENDING:
        s = _PENDING.pop()
        torch.cuda.current_stream(s.device).wait_stream(s)
    _HELD.clear()  # after the waits: the blocks return to the allocator in compute-stream order


def on_side(t: torch.Tensor) -> bool:
    return WGRAD_STREAM and t.is_cuda and not torch.cuda.is_current_stream_capturing()


def ready_event(t: torch.Tensor, enabled: bool = True):
    """An event on the compute stream at this point (for a side launch enqueued later that must not wait for the work
    enqueued in between), or None when the side stream is not in use."""
    if not enabled or not on_side(t):
        return None
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    return ev


def launch(fn, *operands, enabled: bool = True, ready=None):
    """Run ``fn()`` (kernel launches that only accumulate into persistent gradient buffers) on the side stream when
    ``enabled`` and ``on_side`` hold for the first operand, else in place; the operands stay allocated until the
    next join (see the module docstring). ``ready``: an event from ``ready_event`` to wait for instead of the compute
    stream's current point."""
    if not enabled or not operands or not on_side(operands[0]):
        fn()
        return
    dev = operands[0].device
    cur = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    if ready is None:
        side.wait_stream(cur)
    else:
        side.wait_event(ready)
    with torch.cuda.stream(side):
        fn()
    # the caching allocator must not hand these to the compute stream before the side is done
    if HOLD:
        _HELD.extend(operands)
    else:
        for t in operands:
            t.record_stream(side)
    if not _PENDING:  # first side launch of this backward pass: join when the pass ends
        torch.autograd.Variable._execution_engine.queue_callback(join_side_streams)
    if side not in _PENDING:
        _PENDING.append(side)
