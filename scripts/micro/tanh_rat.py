"""Accuracy of the rational f32 tanh (common.h tanh_rat) in simulated f32
arithmetic (each fma / product rounded to f32 once; the quotient exact, so
the hardware rcp adds <= 1 ulp on top), in ulp of the correctly rounded
tanh, over 5M arguments."""
import numpy as np

f32 = np.float32
A = [4.89352455891786e-03, 6.37261928875436e-04, 1.48572235717979e-05, 5.12229709037114e-08,
     -8.60467152213735e-11, 2.00018790482477e-13, -2.76076847742355e-16]
B = [4.89352518554385e-03, 2.26843463243900e-03, 1.18534705686654e-04, 1.19825839466702e-06]
C = 7.90531110763549805


def fma(a, b, c):
    return (a.astype(np.float64) * b + c).astype(f32)


def tanh_rat(x):
    x = np.clip(x, f32(-C), f32(C)).astype(f32)
    s = (x * x).astype(f32)
    p = np.full_like(s, f32(A[-1]))
    for a in A[-2::-1]:
        p = fma(s, p, f32(a))
    q = np.full_like(s, f32(B[-1]))
    for b in B[-2::-1]:
        q = fma(s, q, f32(b))
    return ((x * p).astype(f32).astype(np.float64) / q).astype(f32)


rng = np.random.default_rng(0)
xs = np.concatenate([rng.uniform(-10, 10, 2_000_000), rng.uniform(-1, 1, 2_000_000),
                     10 ** rng.uniform(-8, 0, 1_000_000)]).astype(f32)
ref = np.tanh(xs.astype(np.float64))
err = np.abs(tanh_rat(xs).astype(np.float64) - ref) / np.spacing(np.abs(ref).astype(f32))
print(f"max {err.max():.2f} ulp at x = {xs[err.argmax()]:.6g}, mean {err.mean():.3f} ulp")
