"""Restatement of commons-math3 3.4.1 MersenneTwister + BitsStreamGenerator.nextGaussian (test helper).

The reference's Scala tests seed `new MersenneTwister(10L)` etc. (ARIMASuite.scala:44, 77, 100, 115, ...).
MersenneTwister(long seed) -> setSeed(int[]{(int)(seed >>> 32), (int)(seed & 0xffffffffL)}) = MT19937
init_by_array; next(bits) = tempered output >>> (32 - bits); nextDouble = ((next(26) << 26) | next(26)) * 2^-52;
nextGaussian = Box-Muller pair (x, y): alpha = 2*pi*x, r = sqrt(-2*log(y)), returns r*cos(alpha) then r*sin(alpha).
FastMath.log/cos/sin may differ from Python's libm in the last ulp; the series built from these numbers only feed
the reference's tolerance tests (0.01-0.1), so that is immaterial.
"""
import math


class MersenneTwister:
    N, M = 624, 397

    def __init__(self, seed):
        seed &= 0xFFFFFFFFFFFFFFFF
        self._init_by_array([(seed >> 32) & 0xFFFFFFFF, seed & 0xFFFFFFFF])
        self._next_gaussian = None

    def _init_genrand(self, s):
        mt = [0] * self.N
        mt[0] = s & 0xFFFFFFFF
        for i in range(1, self.N):
            mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.mt = mt
        self.mti = self.N

    def _init_by_array(self, key):
        self._init_genrand(19650218)
        mt, N = self.mt, self.N
        i, j = 1, 0
        k = max(N, len(key))
        for _ in range(k):
            mt[i] = ((mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525)) + key[j] + j) & 0xFFFFFFFF
            i += 1
            j += 1
            if i >= N:
                mt[0] = mt[N - 1]
                i = 1
            if j >= len(key):
                j = 0
        for _ in range(N - 1):
            mt[i] = ((mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941)) - i) & 0xFFFFFFFF
            i += 1
            if i >= N:
                mt[0] = mt[N - 1]
                i = 1
        mt[0] = 0x80000000

    def _next32(self):
        N, M = self.N, self.M
        mt = self.mt
        if self.mti >= N:
            for kk in range(N):
                y = (mt[kk] & 0x80000000) | (mt[(kk + 1) % N] & 0x7FFFFFFF)
                mt[kk] = mt[(kk + M) % N] ^ (y >> 1) ^ (0x9908B0DF if (y & 1) else 0)
            self.mti = 0
        y = mt[self.mti]
        self.mti += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF

    def next_bits(self, bits):
        return self._next32() >> (32 - bits)

    def next_double(self):
        high = self.next_bits(26) << 26
        low = self.next_bits(26)
        return (high | low) * 2.0 ** -52

    def next_gaussian(self):
        if self._next_gaussian is None:
            x = self.next_double()
            y = self.next_double()
            alpha = 2 * math.pi * x
            r = math.sqrt(-2 * math.log(y))
            self._next_gaussian = r * math.sin(alpha)
            return r * math.cos(alpha)
        v = self._next_gaussian
        self._next_gaussian = None
        return v

    def gaussians(self, n):
        return [self.next_gaussian() for _ in range(n)]
