"""CPU: the stream-K partition of gemm_pingpong_kernel<..., SKM> and the
contributor lookup of splitk_sk_reduce_kernel (csrc/gemm_pingpong.hpp),
restated in integer arithmetic exactly as the kernels compute it: every
(tile, k-tile) iteration is owned by exactly one (block, segment), no block
has more than two segments, and the fix-up finds each tile's contributors
(in k order) with the right slots."""
import random


def partition(count, KT, G):
    I = count * KT
    owner = {}
    for g in range(G):
        it, it1 = g * I // G, (g + 1) * I // G
        seg = 0
        while seg < 2 and it < it1:  # the kernel's two straight-line segments
            lt = it // KT
            k0 = it - lt * KT
            nk = min(KT - k0, it1 - it)
            for k in range(k0, k0 + nk):
                assert (lt, k) not in owner
                owner[(lt, k)] = (g, seg)
            it += nk
            seg += 1
        assert it == it1, "a block's range spans more than two tiles"
    return owner


def contributors(lt, count, KT, G):
    I = count * KT
    x0, x1 = lt * KT, lt * KT + KT - 1
    b0, b1 = ((x0 + 1) * G - 1) // I, ((x1 + 1) * G - 1) // I
    return [(b, 1 if b * I // G < x0 else 0) for b in range(b0, b1 + 1)]


def test_stream_k_partition_and_fixup():
    rng = random.Random(0)
    cases = [(70, 80, 256), (140, 80, 256), (210, 80, 256), (10, 400, 256), (24, 80, 256), (3, 2, 6), (1, 80, 80)]
    for _ in range(400):
        KT = rng.choice([2, 8, 40, 64, 80, 400])
        count = rng.randint(1, 255)
        cases.append((count, KT, min(256, count * KT)))
    for count, KT, G in cases:
        assert G >= count
        owner = partition(count, KT, G)
        assert len(owner) == count * KT
        for lt in range(count):
            want = sorted({owner[(lt, k)] for k in range(KT)})
            assert contributors(lt, count, KT, G) == want, (count, KT, G, lt)
