#!/usr/bin/env python3
"""Fit / verify the fast fp32 tanh used by the MLP kernels (csrc/mlp_common.h: fast_tanh).

tanh(x) = x + x^3 * P(x^2) on |x| < 0.6 (P: 5 coefficients, relative-error weighted least squares
iterated toward minimax), else 1 - 2 / (exp2(2|x| log2 e) + 1).  Evaluated here in float32 with
numpy's correctly rounded exp2/reciprocal (the GPU's v_exp_f32 / v_rcp_f32 are ~1 ulp); prints the
max relative error against float64 tanh.
"""
import numpy as np

T, N = 0.6, 5


def fit():
    xs = np.cos(np.pi * (np.arange(4000) + 0.5) / 4000) * T / 2 + T / 2
    xs = xs[xs > 1e-4]
    y = np.tanh(xs)
    A = np.stack([xs ** (3 + 2 * k) for k in range(N)], 1)
    w = 1 / np.abs(y)
    c = np.linalg.lstsq(A * w[:, None], (y - xs) * w, rcond=None)[0]
    for _ in range(30):
        r = (xs + A @ c - y) / y
        w2 = w * (1 + 50 * np.abs(r) / np.abs(r).max())
        c = np.linalg.lstsq(A * w2[:, None], (y - xs) * w2, rcond=None)[0]
    return c.astype(np.float32)


def fast_tanh(x, c):
    x = x.astype(np.float32)
    ax = np.abs(x)
    e = np.exp2(ax * np.float32(2.885390081777927)).astype(np.float32)
    big = (np.float32(1) - np.float32(2) * (np.float32(1) / (e + np.float32(1)))).astype(np.float32)
    x2 = (x * x).astype(np.float32)
    p = c[-1]
    for k in range(N - 2, -1, -1):
        p = (p * x2 + c[k]).astype(np.float32)
    small = (x + (x * x2).astype(np.float32) * p).astype(np.float32)
    return np.where(ax < np.float32(T), small, np.copysign(big, x)).astype(np.float32)


if __name__ == "__main__":
    c = fit()
    print("coefficients x^3..x^11:", [float(v) for v in c])
    xx = np.concatenate([np.linspace(-12, 12, 2000001), np.logspace(-8, 1, 100000),
                         -np.logspace(-8, 1, 100000)]).astype(np.float32)
    ref = np.tanh(xx.astype(np.float64))
    rel = np.abs(fast_tanh(xx, c).astype(np.float64) - ref) / np.maximum(np.abs(ref), 1e-30)
    print(f"max relative error {rel.max():.3e} at x = {xx[np.argmax(rel)]}")
