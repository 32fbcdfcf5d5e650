"""Stratified sub-pixel jitter table for subdivision_level > 1: mirror of
compute_jitters (src/bindings/uniform.rs:254-277), uploaded with the uniforms
(UniformGpu::update_buffer, :163-175) and read by project.wgsl /
w6e1.wgsl get_camera_ray as jitter[sample].

The reference draws from rand_pcg 0.3.1's Lcg64Xsh32::new(0, 0) through rand
0.8.5's Rng::gen_range(0.0..1.0) on f64.  Neither crate is in the checkout;
their published algorithms are restated here:
  * Lcg64Xsh32 = PCG32 (64-bit LCG, XSH-RR output): new(state, stream) sets
    increment = 2*stream + 1, state += increment, then one step; next_u32
    outputs from the pre-step state.  Pinned by the PCG reference vector
    (Lcg64Xsh32::new(42, 54) -> 0xa15c02b7, 0x7b47f409, ...; tests/test_jitter.py).
  * next_u64 = two next_u32 calls, low word first (rand_core next_u64_via_u32).
  * gen_range(0.0..1.0) for f64 (UniformFloat::sample_single): 52 high bits
    of next_u64 as the mantissa of a value in [1, 2), minus 1, times the
    range width (1), plus the low end (0).
The f64 -> f32 rounding of each jitter is the reference's `as f32`.
"""
import numpy as np

MAX_SUBDIVISION = 10   # src/bindings/uniform.rs:36
_MASK64 = (1 << 64) - 1
_MULT = 6364136223846793005


class Lcg64Xsh32:
    def __init__(self, state, stream):
        self.increment = ((stream << 1) | 1) & _MASK64
        self.state = (state + self.increment) & _MASK64
        self._step()

    def _step(self):
        self.state = (self.state * _MULT + self.increment) & _MASK64

    def next_u32(self):
        s = self.state
        self._step()
        rot = s >> 59
        xsh = (((s >> 18) ^ s) >> 27) & 0xFFFFFFFF
        return ((xsh >> rot) | (xsh << ((32 - rot) & 31))) & 0xFFFFFFFF

    def next_u64(self):
        lo = self.next_u32()
        hi = self.next_u32()
        return (hi << 32) | lo

    def gen_unit_f64(self):
        bits = (self.next_u64() >> 12) | 0x3FF0000000000000
        v12 = np.array([bits], np.uint64).view(np.float64)[0]
        return float(v12) - 1.0


def compute_jitters(pixel_size, subdivs):
    """[subdivs^2, 2] float32: row-major over (i = row, j = column) strata."""
    if not (0 < subdivs <= MAX_SUBDIVISION) or pixel_size == 0.0:
        raise ValueError("subdivs must be in 1..10 and pixel_size nonzero")
    if subdivs == 1:
        return np.zeros((1, 2), np.float32)
    rng = Lcg64Xsh32(0, 0)
    step = pixel_size / subdivs
    out = []
    for i in range(subdivs):
        for j in range(subdivs):
            u1 = rng.gen_unit_f64()
            u2 = rng.gen_unit_f64()
            out.append(((u1 + j) * step - pixel_size * 0.5, (u2 + i) * step - pixel_size * 0.5))
    return np.array(out, np.float64).astype(np.float32)


def jitters_for(height, subdivs):
    """The table UniformGpu::update_buffer uploads: pixel_size = 1 / H."""
    return compute_jitters(1.0 / float(height), subdivs)
