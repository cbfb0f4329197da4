"""CPU pins of the oracle's G2 arithmetic (used to check ParamsKZG's g2 / s_g2):
the standard generator lies on the twist y^2 = x^3 + 3/(9+u), has order r, and the
group law agrees with scalar multiplication."""
import bn254_ref as B


def test_g2_generator_on_twist_and_order_r():
    assert B.g2_on_curve(B.G2_GEN)
    assert B.g2_mul(B.G2_GEN, B.R) is None
    assert B.g2_mul(B.G2_GEN, B.R - 1) == (B.G2_GEN[0], ((-B.G2_GEN[1][0]) % B.P, (-B.G2_GEN[1][1]) % B.P))


def test_g2_group_law():
    a, b = 0x1234567, 0xABCDEF0123
    pa, pb = B.g2_mul(B.G2_GEN, a), B.g2_mul(B.G2_GEN, b)
    assert B.g2_on_curve(pa) and B.g2_on_curve(pb)
    assert B.g2_add(pa, pb) == B.g2_mul(B.G2_GEN, a + b)
    assert B.g2_add(pa, pa) == B.g2_mul(B.G2_GEN, 2 * a)


def test_g2_raw_layout():
    limbs = B.g2_affine_mont_limbs(B.G2_GEN)
    assert len(limbs) == 16 and B.g2_affine_mont_limbs(None) == [0] * 16
    assert limbs[:4] == B.fq_mont_limbs(B.G2_GEN[0][0]) and limbs[4:8] == B.fq_mont_limbs(B.G2_GEN[0][1])
