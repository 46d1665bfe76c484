"""Java 8 Float.toString / Double.toString (sun.misc.FloatingDecimal, the JDK the reference targets;
outside /root/reference), restated from the published algorithm for the tests: the check on the
engine's (siddhi_amd/csrc/chm_order.h java_value_of_float/_double) and the oracle's restatements.
String.valueOf of a float / double partition key is this text (ValuePartitionExecutor.java:34-40).

dtoa: the easy case (an integer value that fits a long: its decimal digits, trailing zeros dropped,
low digits rounded away past the float's precision), else Steele & White digit generation with the
JDK's stopping test (low: B < M, high: B + M > 10S -- >= in the big-integer path) in 32-bit, 64-bit
or unbounded arithmetic, with the 32/64-bit paths' overflow of M reproduced, then the last digit
rounded by the stopping condition (roundup keeps the digit count: "0.0020"-style outputs)."""
import struct

N_5_BITS = [0, 3, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28, 31, 33, 35, 38, 40, 42, 45, 47, 49, 52, 54, 56, 59, 61]
INSIG = [0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 8, 8, 8, 9, 9, 9, 9,
         10, 10, 10, 11, 11, 11, 12, 12, 12, 12, 13, 13, 13, 14, 14, 14, 15, 15, 15, 15, 16, 16, 16, 17, 17, 17,
         18, 18, 18, 19]


def _wrap(v, bits):
    m = 1 << bits
    v &= m - 1
    return v - m if v >= m >> 1 else v


def _est_dec_exp(fract_bits, bin_exp):
    d2 = struct.unpack("<d", struct.pack("<q", 0x3FF0000000000000 | (fract_bits & 0xFFFFFFFFFFFFF)))[0]
    d = (d2 - 1.5) * 0.289529654 + 0.176091259 + bin_exp * 0.301029995663981
    import math
    return math.floor(d)


def _dtoa(bin_exp, fract_bits, n_sig):
    """-> (digits list of ints, decExponent)"""
    tail_zeros = (fract_bits & -fract_bits).bit_length() - 1
    n_fract_bits = 53 - tail_zeros
    n_tiny = max(0, n_fract_bits - bin_exp - 1)
    if -21 <= bin_exp <= 62 and n_tiny < 27 and n_fract_bits + N_5_BITS[n_tiny] < 64 and n_tiny == 0:
        insignificant = INSIG[bin_exp - n_sig - 1] if (bin_exp > n_sig and 1 < bin_exp - n_sig - 1 < 64) else 0
        lv = fract_bits << (bin_exp - 52) if bin_exp >= 52 else fract_bits >> (52 - bin_exp)
        dec_exp = 0
        if insignificant:
            p10 = 10 ** insignificant
            residue = lv % p10
            lv //= p10
            dec_exp += insignificant
            if residue >= p10 >> 1:
                lv += 1
        s = str(lv)
        stripped = s.rstrip("0")
        dec_exp += len(s) - len(stripped)
        digits = [int(c) for c in stripped]
        return digits, dec_exp + len(digits)
    dec_exp = _est_dec_exp(fract_bits, bin_exp)
    B5 = max(0, -dec_exp)
    B2 = B5 + n_tiny + bin_exp
    S5 = max(0, dec_exp)
    S2 = S5 + n_tiny
    M5 = B5
    M2 = B2 - n_sig
    fract_bits >>= tail_zeros
    B2 -= n_fract_bits - 1
    c2 = min(B2, S2)
    B2 -= c2
    S2 -= c2
    M2 -= c2
    if n_fract_bits == 1:
        M2 -= 1
    if M2 < 0:
        B2 -= M2
        S2 -= M2
        M2 = 0
    b_bits = n_fract_bits + B2 + (N_5_BITS[B5] if B5 < 27 else B5 * 3)
    ten_s_bits = S2 + 1 + (N_5_BITS[S5 + 1] if S5 + 1 < 27 else (S5 + 1) * 3)
    digits = []
    if b_bits < 64 and ten_s_bits < 64:
        bits = 32 if (b_bits < 32 and ten_s_bits < 32) else 64
        b = _wrap(fract_bits * 5 ** B5, bits) << B2
        b = _wrap(b, bits)
        s = _wrap(5 ** S5 << S2, bits)
        m = _wrap(5 ** M5 << M2, bits)
        tens = _wrap(s * 10, bits)
        q = b // s
        b = _wrap(10 * (b % s), bits)
        m = _wrap(m * 10, bits)
        low = b < m
        high = _wrap(b + m, bits) > tens
        if q == 0 and not high:
            dec_exp -= 1
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:
            high = low = False
        while not low and not high:
            q = b // s
            b = _wrap(10 * (b % s), bits)
            m = _wrap(m * 10, bits)
            if m > 0:
                low = b < m
                high = _wrap(b + m, bits) > tens
            else:
                low = high = True
            digits.append(q)
        low_diff = _wrap(_wrap(b << 1, bits) - tens, bits)
    else:
        Bv = fract_bits * 5 ** B5 << B2
        Sv = 5 ** S5 << S2
        Mv = 5 ** (M5 + 1) << (M2 + 1)
        tenS = 5 ** (S5 + 1) << (S2 + 1)
        q, Bv = divmod(Bv, Sv)
        Bv *= 10
        low = Bv < Mv
        high = Bv + Mv >= tenS
        if q == 0 and not high:
            dec_exp -= 1
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:
            high = low = False
        while not low and not high:
            q, Bv = divmod(Bv, Sv)
            Bv *= 10
            Mv *= 10
            low = Bv < Mv
            high = Bv + Mv >= tenS
            digits.append(q)
        low_diff = ((Bv << 1) > tenS) - ((Bv << 1) < tenS) if (high and low) else 0
    dec_exponent = dec_exp + 1
    if high:
        if low:
            if low_diff == 0:
                if digits[-1] & 1:
                    dec_exponent = _roundup(digits, dec_exponent)
            elif low_diff > 0:
                dec_exponent = _roundup(digits, dec_exponent)
        else:
            dec_exponent = _roundup(digits, dec_exponent)
    return digits, dec_exponent


def _roundup(digits, dec_exponent):
    i = len(digits) - 1
    q = digits[i]
    if q == 9:
        while q == 9 and i > 0:
            digits[i] = 0
            i -= 1
            q = digits[i]
        if q == 9:
            digits[0] = 1
            return dec_exponent + 1
    digits[i] = q + 1
    return dec_exponent


def _format(neg, digits, e):
    d = "".join(str(x) for x in digits)
    out = "-" if neg else ""
    n = len(d)
    if 0 < e < 8:
        c = min(n, e)
        out += d[:c]
        if c < e:
            out += "0" * (e - c) + ".0"
        else:
            out += "." + (d[c:] if c < n else "0")
    elif -3 < e <= 0:
        out += "0." + "0" * (-e) + d
    else:
        out += d[0] + "." + (d[1:] if n > 1 else "0") + "E"
        out += ("-" + str(-e + 1)) if e <= 0 else str(e - 1)
    return out


def double_to_string(bits: int) -> str:
    """Double.toString of the double with these raw 64 bits."""
    bits &= (1 << 64) - 1
    neg = bits >> 63 != 0
    fract = bits & ((1 << 52) - 1)
    be = (bits >> 52) & 0x7FF
    if be == 0x7FF:
        return ("-Infinity" if neg else "Infinity") if fract == 0 else "NaN"
    if be == 0:
        if fract == 0:
            return "-0.0" if neg else "0.0"
        lz = 64 - fract.bit_length()
        shift = lz - 11
        fract <<= shift
        be = 1 - shift
        n_sig = 64 - lz
    else:
        fract |= 1 << 52
        n_sig = 53
    be -= 1023
    digits, e = _dtoa(be, fract, n_sig)
    return _format(neg, digits, e)


def float_to_string(bits: int) -> str:
    """Float.toString of the float with these raw 32 bits."""
    bits &= 0xFFFFFFFF
    neg = bits >> 31 != 0
    fract = bits & ((1 << 23) - 1)
    be = (bits >> 23) & 0xFF
    if be == 0xFF:
        return ("-Infinity" if neg else "Infinity") if fract == 0 else "NaN"
    if be == 0:
        if fract == 0:
            return "-0.0" if neg else "0.0"
        lz = 32 - fract.bit_length()
        shift = lz - 8
        fract <<= shift
        be = 1 - shift
        n_sig = 32 - lz
    else:
        fract |= 1 << 23
        n_sig = 24
    be -= 127
    digits, e = _dtoa(be, fract << 29, n_sig)
    return _format(neg, digits, e)


def f32(x: float) -> int:
    return struct.unpack("<I", struct.pack("<f", x))[0]


def f64(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]
