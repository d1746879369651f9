"""Host-side check of the row-walking pooled conv's LDS ring size (ore_conv_pool.hip, cp_nring).

The kernel walks the conv output plane in steps of S quads (4 output columns each, qrow quads per
conv row), max-reduces every step's values into pooled rows held in `nring` LDS slots (pooled row
py in slot py % nring), and after each step's barrier stores and clears the pooled rows whose three
conv rows are done.  Without a second barrier the clears race with the NEXT step's maxima, so the
ring must be large enough that (a) no two live pooled rows share a slot and (b) no slot cleared
after a step is touched by the next one.  This restates the kernel's step / flush rules and checks
the closed form nring = ((qrow + 2 S - 2) / qrow + 4) / 2 against the exact requirement."""
import pytest


def ring_need(qrow, Ho, S, race_free=True, bands=1):
    """Smallest ring for which the walk of every band has no slot conflict (the kernel's rules)."""
    Hp = (Ho - 3) // 2 + 1
    pbn = (Hp + bands - 1) // bands
    need = 2
    for band in range(bands):
        py0, py1 = band * pbn, min(band * pbn + pbn, Hp)
        if py0 >= py1:
            continue
        q0, nq = 2 * py0 * qrow, min(2 * py1 + 1, Ho) * qrow
        for nr in range(need, 512):
            owner, cleared, py_next, ok = {}, set(), py0, True
            for qs in range(q0, nq, S):
                qe = min(qs + S, nq)
                for qd in range(qs, qe):
                    oy = qd // qrow
                    pa = oy >> 1
                    pb = pa - 1 if (oy % 2 == 0 and oy >= 2) else -1
                    for py in (pa, pb):
                        if not py0 <= py < py1:
                            continue
                        s = py % nr
                        if owner.get(s, py) != py or (race_free and s in cleared):
                            ok = False
                        owner[s] = py
                rd = qe // qrow
                pe = py1 if qe == nq else (((rd - 3) >> 1) + 1 if rd >= 3 else 0)
                pe = min(pe, py1)
                cleared = set()
                for py in range(py_next, pe):
                    cleared.add(py % nr)
                    if owner.get(py % nr) == py:
                        del owner[py % nr]
                py_next = max(py_next, pe)
                if not ok:
                    break
            if ok:
                need = nr
                break
    return need


def nring_closed_form(qrow, S):
    return ((qrow + 2 * S - 2) // qrow + 4) // 2


@pytest.mark.parametrize("S", [64, 128])
def test_closed_form_covers_the_walk(S):
    for Wo in range(6, 230, 7):
        qrow = (Wo + 3) // 4
        nr = nring_closed_form(qrow, S)
        for Ho in range(5, 230, 23):
            assert ring_need(qrow, Ho, S) <= nr, (S, qrow, Ho, nr)


def test_conv1_ring_sizes():
    # conv1 (109 x 109 -> pool1 54 x 54, 28 quads per row): the sizes the kernel allocates
    assert nring_closed_form(28, 64) == 4 and ring_need(28, 109, 64) == 4
    assert nring_closed_form(28, 128) == 7 and ring_need(28, 109, 128) <= 7
    # the double-barrier variant (2 bands, clears separated from the next step's maxima)
    assert ring_need(28, 109, 64, race_free=False, bands=2) == 3
