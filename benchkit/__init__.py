"""Measurement infrastructure of bench.py (the CPU baseline, the roofline
fields, the self-launcher, failure containment, the one-GPU rehearsal's
stand-in communicator).  Not part of the product path: sfl_amd/ never
imports it."""
