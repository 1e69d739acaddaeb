"""Coefficients of the shading's short f64 atan core (bh_crmath.hpp, atan2_core): atan(u) = u + u^3 P(u^2)
for |u| <= tan(pi/8), P an 11-term Chebyshev fit of (atan(sqrt s) - sqrt s) / s^1.5 on [0, tan^2(pi/8)]
(mpmath, 60 digits), printed as C hex literals, with the fit's error and a dense check of the f64
evaluation against mpmath.

    python tools/atan2_coefs.py"""
import random

import mpmath as mp


def main():
    mp.mp.dps = 60
    smax = mp.tan(mp.pi / 8) ** 2

    def P(s):
        if s == 0:
            return mp.mpf(-1) / 3
        r = mp.sqrt(s)
        return (mp.atan(r) - r) / (s * r)

    poly, err = mp.chebyfit(P, [0, smax], 11, error=True)
    coefs = [float(c) for c in poly]  # highest degree first
    print("ATAN_P[11] = {" + ", ".join(c.hex() for c in coefs) + "}")
    print("fit error on P:", mp.nstr(err, 5), " relative error on atan <=", mp.nstr(err * smax, 5),
          "= 2^" + mp.nstr(mp.log(err * smax, 2), 4))
    worst = mp.mpf(0)
    rng = random.Random(1)
    umax = float(mp.tan(mp.pi / 8))
    for i in range(200000):
        u = rng.uniform(0, umax) if i > 3 else [1e-300, 1e-8, umax, 0.2][i]
        s = u * u
        p = coefs[0]
        for c in coefs[1:]:
            p = p * s + c
        a = u + (u * s) * p
        t = mp.atan(mp.mpf(u))
        worst = max(worst, abs((mp.mpf(a) - t) / t))
    print("f64 evaluation (no FMA), worst relative error: 2^" + mp.nstr(mp.log(worst, 2), 4))


if __name__ == "__main__":
    main()
