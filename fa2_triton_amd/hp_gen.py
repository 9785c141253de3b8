"""Generator of the hand-placed CDNA4 (gfx950) instruction streams of the forward kernel.

The hot loop of `fwd_hp_kernel` (csrc/fwd_hp_kernel.h) is not compiler-scheduled: this module
writes it as one inline-asm statement per (dtype, causal) variant into csrc/gen/fwd_hp_body.h
(build.py calls `write_headers()` before compiling).  Every MFMA, exponential, LDS read, LDS-DMA
piece and wait is placed by the tables below, in the spirit of cdna_hip_programming.md
"4-wave, one-wave-per-SIMD, persistent structure": each 32-cycle MFMA gap carries a planned set
of single-issue fillers (issue costs summed per gap, at most two exponentials), reads are
counted (`s_waitcnt lgkmcnt(N)` computed from the exact LDS issue order), and every register
hazard the hardware does not interlock (MFMA result -> vector read, vector write -> MFMA operand,
transcendental -> use, permlane source) is padded by the `Emitter` from a register-state model,
so the schedule tables only decide the ORDER.

Algorithm (same as the reference's compute_row_block, /root/reference/src/forward/
compute_row_blocks.py:38-103, and fwd_pipe_kernel): per 64-key tile, S^T = K Q^T (swapped so the
softmax row is one lane pair), online softmax in base 2 with defer-max (running max moved only
when a row grows by more than 8), O^T += V^T P^T.  Differences of arrangement only:
  * Q is pre-scaled by softmax_scale * log2(e) (rounded once to the input dtype) and the S chain
    starts from -m_ref (the running reference max) as its initial accumulator, so the MFMA chain
    yields the exponent argument z directly: no per-score multiply-add;
  * the row sums of P are added in the PV phase (where the VALU has room), the exponentials of a
    tile ride on the next tile's QK^T MFMAs.
"""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
GEN = os.path.join(HERE, "csrc", "gen")

NINF = "0xff800000"


def _regs(spec):
    """'v[3:5]' / 'a7' / 's[64:65]' -> ['v3', 'v4', 'v5'] ..."""
    spec = spec.strip()
    m = re.fullmatch(r"([vas])\[(\d+):(\d+)\]", spec)
    if m:
        return [f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    m = re.fullmatch(r"([vas])(\d+)", spec)
    if m:
        return [spec]
    return []  # operands (%[..]), constants, literals: not tracked


def rng(kind, base, n):
    return f"{kind}{base}" if n == 1 else f"{kind}[{base}:{base + n - 1}]"


class Emitter:
    """Straight-line instruction emitter with a hazard / LDS-wait model.

    Wait states are counted per issued instruction (s_nop N = N + 1), the unit of the hazard
    tables; the values below carry margin over the gfx950 minima (8-pass XDL result -> vector
    read 12, vector write -> MFMA operand 2, transcendental -> use 1, VALU -> permlane 2)."""

    MFMA_RESULT = 18   # MFMA writes r  -> any non-chain access of r
    TO_MFMA = 3        # VALU / accvgpr_write writes r -> MFMA reads r
    TRANS_USE = 2      # v_exp writes r -> vector use
    TO_PERM = 3        # VALU writes r -> v_permlane32_swap reads r
    MFMA_READ_WAR = 4  # MFMA reads r (A/B) -> something writes r
    MFMA_C_WAR = 18    # MFMA reads r as C -> something writes r
    M0_DMA = 2         # s_* writes m0 -> LDS-DMA

    def __init__(self):
        self.out = []
        self.ws = 0
        self.wr = {}       # reg -> (ws, kind)
        self.rd_ab = {}    # reg -> ws of the last MFMA A/B read
        self.rd_c = {}     # reg -> ws of the last MFMA C read
        self.ds = []       # pending LDS reads, oldest first: sets of destination regs
        self.n_mfma = 0

    # -- bookkeeping -------------------------------------------------------------------------
    def _line(self, text, ws=1):
        self.out.append(text)
        self.ws += ws

    def reset(self):
        """Block boundary after a barrier / wait: every producer is long done (the barrier waits
        far longer than any hazard window) and no LDS read is pending."""
        assert not self.ds, "LDS reads pending across a block boundary"
        self.wr.clear()
        self.rd_ab.clear()
        self.rd_c.clear()

    def _need_lgkm(self, regs):
        hit = -1
        for j, dst in enumerate(self.ds):
            if dst & regs:
                hit = j
        if hit >= 0:
            n = len(self.ds) - 1 - hit
            assert n <= 15
            self._line(f"s_waitcnt lgkmcnt({n})")
            self.ds = self.ds[hit + 1:]

    def _pad(self, need):
        need = max(need, 0)
        while need > 0:
            k = min(need, 16)
            self._line(f"s_nop {k - 1}", k)
            need -= k

    def _hazards(self, kind, reads, writes, c_regs=(), chain=False):
        need = 0
        for r in reads | writes:
            w = self.wr.get(r)
            if w is None:
                continue
            dist = self.ws - w[0]
            pk = w[1]
            if pk == "mfma":
                if kind == "mfma" and chain and r in c_regs:
                    continue
                need = max(need, self.MFMA_RESULT - dist)
                continue
            if kind == "mfma" and r in reads:
                need = max(need, self.TO_MFMA - dist)
            if pk == "trans" and r in reads:
                need = max(need, self.TRANS_USE - dist)
            if kind == "perm" and pk in ("valu", "trans", "accr") and r in reads:
                need = max(need, self.TO_PERM - dist)
            if pk == "m0" and kind == "dma":
                need = max(need, self.M0_DMA - dist)
        for r in writes:
            if kind == "mfma" and chain:
                break
            if r in self.rd_ab:
                need = max(need, self.MFMA_READ_WAR - (self.ws - self.rd_ab[r]))
            if r in self.rd_c:
                need = max(need, self.MFMA_C_WAR - (self.ws - self.rd_c[r]))
        self._pad(need)

    def _commit(self, kind, writes):
        for r in writes:
            self.wr[r] = (self.ws, kind)

    # -- instructions ------------------------------------------------------------------------
    def mfma(self, op, d, a, b, c):
        rd, ra, rb, rc = map(set, map(_regs, (d, a, b, c)))
        chain = rc == rd
        self._need_lgkm(ra | rb | rc | rd)
        self._hazards("mfma", ra | rb | rc, rd, c_regs=rc, chain=chain)
        for r in ra | rb:
            self.rd_ab[r] = self.ws
        for r in rc:
            self.rd_c[r] = self.ws
        self._commit("mfma", rd)
        self._line(f"{op} {d}, {a}, {b}, {c}")
        self.n_mfma += 1

    def valu(self, text, dst, srcs=(), kind="valu"):
        wr = set()
        for d in ([dst] if isinstance(dst, str) else (dst or [])):
            wr |= set(_regs(d))
        rd = set()
        for s in srcs:
            rd |= set(_regs(s))
        self._need_lgkm(rd | wr)
        self._hazards(kind, rd, wr)
        self._line(text)
        self._commit(kind, wr)

    def ds_read(self, text, dst, addr=None):
        wr = set(_regs(dst))
        self._need_lgkm(wr)
        self._hazards("ds", set(_regs(addr)) if addr else set(), wr)
        self._line(text)
        self.ds.append(wr)

    def salu(self, text, m0=False):
        self._line(text)
        if m0:
            self.wr["m0"] = (self.ws, "m0")

    def dma(self, text):
        self._hazards("dma", {"m0"}, set())
        self._line(text)

    def raw(self, text, ws=1):
        self._line(text, ws)

    def label(self, name):
        self.out.append(f"{name}:")

    def drain_lds(self):
        if self.ds:
            self._line("s_waitcnt lgkmcnt(0)")
            self.ds = []

    def drain_mfma(self):
        """Pad until every MFMA result may be read by any instruction."""
        need = 0
        for r, (w, k) in self.wr.items():
            if k == "mfma":
                need = max(need, self.MFMA_RESULT - (self.ws - w))
        self._pad(need)


# ----------------------------------------------------------------------------------------------
# Register map of the forward (fixed registers owned by the asm statement)
#   v[0:127]    S[set][rb][t] scores / exponent arguments / probabilities (16 per key half)
#   v[128:159]  PF[rb][kk] packed P (B operand of O^T += V^T P^T), 4 dwords per 16-key step
#   v[160:191]  INIT[rb] = -m_ref broadcast (initial accumulator of the S chains)
#   v[192:215]  row statistics and temporaries
#   a[0:127]    O^T[rb][dt] accumulators
#   a[128:191]  Q fragments (compiler-placed "a" operands %[q0]..%[q15])
#   a[192:207]  K fragment ring (4 slots), a[208:223] V^T fragment ring (4 slots)
#   s[64:91]    scalar state
def S(st, rb, t, i=None):
    base = ((st * 2 + rb) * 2 + t) * 16
    return rng("v", base, 16) if i is None else f"v{base + i}"


def PF(rb, kk, j=None):
    base = 128 + (rb * 4 + kk) * 4
    return rng("v", base, 4) if j is None else f"v{base + j}"


def INIT(rb, j=None):
    return rng("v", 160 + 16 * rb, 16) if j is None else f"v{160 + 16 * rb + j}"


MRUN = ["v192", "v193"]
LSUM = [["v194", "v195"], ["v196", "v197"]]
MREF = ["v198", "v199"]
THR = ["v200", "v201"]
MAH = [["v202", "v203"], ["v204", "v205"]]
MX = ["v206", "v207"]
REL = ["v208", "v209"]
VNINF = "v210"
TMP = ["v211", "v212", "v213", "v214", "v215"]
N_VGPR = 216


def O(rb, dt, i=None):
    base = (rb * 4 + dt) * 16
    return rng("a", base, 16) if i is None else f"a{base + i}"


def KR(slot):
    return rng("a", 192 + 4 * slot, 4)


def VR(slot, half=None):
    base = 208 + 4 * slot
    return rng("a", base, 4) if half is None else rng("a", base + 2 * half, 2)


AGPR_CLOBBER = list(range(0, 128)) + list(range(192, 256))

# scalar state
SI = "s64"        # period index i
SN1 = "s65"       # 64 (i + 1): first key of tile i + 1
SKD = "s[68:71]"  # K descriptor of the tile being requested
SVD = "s[72:75]"  # V descriptor
SKP = ("s76", "s77")  # next K tile to request: byte address
SVP = ("s78", "s79")
SKR = "s80"       # bytes of K from that tile to the end of the slice
SVR = "s81"
SM0 = "s82"       # saved m0
SVOTE = "s[84:85]"
SVOTE2 = "s[86:87]"
SMASK = ["s[88:89]", "s[90:91]"]
SGPR_CLOBBER = list(range(64, 92))

LEADK = 3  # K fragments in flight ahead of their MFMAs
LEADV = 3


def elem_order():
    """The 64 softmax elements (rb, t, i) of a lane in 16-key-step order: kk-major, then rb."""
    out = []
    for kk in range(4):
        for rb in range(2):
            for j in range(8):
                out.append((kk, rb, kk >> 1, (kk & 1) * 8 + j))
    return out


class GapScheduler:
    """Fills the gaps between n MFMAs with filler items.

    An item (stream, cost, release, deadline, emit) may go into gap g (after MFMA g; gap -1 =
    before the first MFMA) once g >= release and its predecessor in the same stream is placed.
    Gap by gap, eligible items are taken earliest-deadline-first while the gap's issue budget
    (32-cycle MFMA gap minus the MFMA's own 8 issue cycles) lasts; an item at its deadline goes in
    regardless.  Costs: v_exp 8, other vector / LDS instructions 4, an LDS-DMA piece 16
    (MI355X_MICROARCH.md, per-instruction issue costs)."""

    BUDGET = 24

    def __init__(self, n):
        self.n = n
        self.items = []

    def add(self, stream, cost, release, deadline, emit):
        self.items.append(dict(stream=stream, cost=cost, rel=release, dl=deadline, emit=emit, seq=len(self.items)))

    def run(self, mfma, pre_budget=0):
        pending = list(self.items)

        def heads():
            seen, out = set(), []
            for it in pending:
                if it["stream"] not in seen:
                    seen.add(it["stream"])
                    out.append(it)
            return out

        last_use = {}
        tick = [0]

        def fill(g, budget):
            while True:
                el = [it for it in heads() if it["rel"] <= g]
                if not el:
                    return
                # earliest deadline first; among equals the stream served longest ago (two
                # dependent chains alternate instead of running back to back)
                el.sort(key=lambda it: (it["dl"], last_use.get(it["stream"], -1), it["seq"]))
                it = el[0]
                if it["cost"] > budget and it["dl"] > g:
                    # something cheaper that fits?
                    fit = [x for x in el if x["cost"] <= budget]
                    if not fit:
                        return
                    it = fit[0]
                pending.remove(it)
                it["emit"]()
                last_use[it["stream"]] = tick[0]
                tick[0] += 1
                budget -= it["cost"]

        fill(-1, pre_budget)
        for g in range(self.n):
            mfma(g)
            fill(g, self.BUDGET)
        while pending:  # no MFMA left to cover them
            it = heads()[0]
            pending.remove(it)
            it["emit"]()


class FwdGen:
    def __init__(self, bf16, causal):
        self.bf16, self.causal = bf16, causal
        self.mop = "v_mfma_f32_32x32x16_bf16" if bf16 else "v_mfma_f32_32x32x16_f16"
        self.cvtop = "v_cvt_pk_bf16_f32" if bf16 else "v_cvt_pk_f16_f32"
        self.e = Emitter()

    # -- pieces ------------------------------------------------------------------------------
    def k_read(self, kbuf, m):
        """K fragment m (key half t = m // 8, k-step ks = m % 8) of the buffer kbuf -> ring."""
        t, ks = m // 8, m % 8
        imm = kbuf * 16384 + (ks >> 1) * 4096 + 32 * t * 64
        base = "%[kb1]" if ks & 1 else "%[kb0]"
        dst = KR(m % 4)
        self.e.ds_read(f"ds_read_b128 {dst}, {base} offset:{imm}", dst)

    def v_read(self, vbuf, m, half):
        """Half `half` of V^T fragment m (kk = m // 4, dt = m % 4) of V buffer vbuf -> ring."""
        kk, dt = m // 4, m % 4
        imm = 32768 + vbuf * 16384 + dt * 4096 + 16 * kk * 64
        base = "%[vb]" if half else "%[va]"
        dst = VR(m % 4, half)
        self.e.ds_read(f"ds_read_b64_tr_b16 {dst}, {base} offset:{imm}", dst)

    def dma_piece(self, which, par, it):
        """LDS-DMA piece `it` of this wave: K(i+2) into K buffer par, V(i+1) into V buffer 1-par."""
        if which == "k":
            imm = par * 16384 + it * 4096
            desc = SKD
        else:
            imm = 32768 + (1 - par) * 16384 + it * 4096
            desc = SVD
        self.e.salu(f"s_add_u32 m0, %[mlds], {imm}", m0=True)
        self.e.dma(f"buffer_load_dwordx4 %[off{it}], {desc}, 0 offen lds")

    def descriptors(self):
        e = self.e
        for (p0, p1), rem, d in ((SKP, SKR, 68), (SVP, SVR, 72)):
            e.salu(f"s_mov_b32 s{d}, {p0}")
            e.salu(f"s_and_b32 s{d + 1}, {p1}, 0xffff")
            e.salu(f"s_max_i32 s{d + 2}, {rem}, 0")
            e.salu(f"s_mov_b32 s{d + 3}, 0x20000")
            e.salu(f"s_add_u32 {p0}, {p0}, %[tileb]")
            e.salu(f"s_addc_u32 {p1}, {p1}, 0")
            e.salu(f"s_sub_i32 {rem}, {rem}, %[tileb]")

    def exp(self, st, el):
        kk, rb, t, i = el
        r = S(st, rb, t, i)
        self.e.valu(f"v_exp_f32 {r}, {r}", r, [r], kind="trans")

    def cvt(self, st, rb, kk, j):
        t, i0 = kk >> 1, (kk & 1) * 8 + 2 * j
        a, b = S(st, rb, t, i0), S(st, rb, t, i0 + 1)
        d = PF(rb, kk, j)
        self.e.valu(f"{self.cvtop} {d}, {a}, {b}", d, [a, b])

    def add(self, st, el, c):
        kk, rb, t, i = el
        r = S(st, rb, t, i)
        l = LSUM[rb][c]
        self.e.valu(f"v_add_f32 {l}, {l}, {r}", l, [l, r])

    def mask_elem(self, st, rb, t, i):
        """z = key offset o < rel[rb] ? z : -inf  (o = 32 t + (i & 3) + 8 (i >> 2))."""
        o = 32 * t + (i & 3) + 8 * (i >> 2)
        r = S(st, rb, t, i)
        sm = SMASK[i & 1]
        e = self.e
        e.valu(f"v_cmp_gt_i32_e64 {sm}, {REL[rb]}, {o}", None, [REL[rb]])
        e.valu(f"v_cndmask_b32_e64 {r}, {VNINF}, {r}, {sm}", r, [r, VNINF])

    # max chain of (rb, half t): 16 values -> 8 instructions
    def max_ops(self, st, rb, t):
        ops = []
        v = [S(st, rb, t, i) for i in range(16)]
        m = MAH[rb][t]
        ops.append((f"v_max3_f32 {m}, {v[0]}, {v[1]}, {v[2]}", m, v[0:3]))
        for k in range(3, 15, 2):
            ops.append((f"v_max3_f32 {m}, {m}, {v[k]}, {v[k + 1]}", m, [m, v[k], v[k + 1]]))
        ops.append((f"v_max_f32 {m}, {m}, {v[15]}", m, [m, v[15]]))
        return ops

    def row_max_finish(self):
        """mx[rb] = max over the lane pair of max(MAH[rb][0], MAH[rb][1])."""
        e = self.e
        for rb in range(2):
            e.valu(f"v_max_f32 {MX[rb]}, {MAH[rb][0]}, {MAH[rb][1]}", MX[rb], MAH[rb])
            e.valu(f"v_mov_b32 {TMP[rb]}, {MX[rb]}", TMP[rb], [MX[rb]])
        for rb in range(2):
            e.valu(f"v_permlane32_swap_b32 {MX[rb]}, {TMP[rb]}", [MX[rb], TMP[rb]], [MX[rb], TMP[rb]], kind="perm")
        for rb in range(2):
            e.valu(f"v_max_f32 {MX[rb]}, {MX[rb]}, {TMP[rb]}", MX[rb], [MX[rb], TMP[rb]])

    def rescale(self, st, lbl_skip=None):
        """Defer-max rescale: for each row block, m_new = max(m_run, mx + m_ref), m_use = m_new or
        0 when -inf; O, l *= exp2(m_run - m_use); z of set st -= m_use - m_ref; INIT = -m_use."""
        e = self.e
        t_new, t_use, t_alpha, t_shift = TMP[0], TMP[1], TMP[2], TMP[3]
        # free during a rescale: the row-max chains and the mask limits (MX is still read)
        scratch = [TMP[4], MAH[0][0], MAH[0][1], MAH[1][0], MAH[1][1], REL[0], REL[1]]
        for rb in range(2):
            e.valu(f"v_add_f32 {t_new}, {MX[rb]}, {MREF[rb]}", t_new, [MX[rb], MREF[rb]])
            e.valu(f"v_max_f32 {t_new}, {MRUN[rb]}, {t_new}", t_new, [MRUN[rb], t_new])
            e.valu(f"v_cmp_eq_f32_e32 vcc, {VNINF}, {t_new}", None, [VNINF, t_new])
            e.valu(f"v_cndmask_b32_e64 {t_use}, {t_new}, 0, vcc", t_use, [t_new])
            e.valu(f"v_sub_f32 {t_alpha}, {MRUN[rb]}, {t_use}", t_alpha, [MRUN[rb], t_use])
            e.valu(f"v_exp_f32 {t_alpha}, {t_alpha}", t_alpha, [t_alpha], kind="trans")
            e.valu(f"v_sub_f32 {t_shift}, {t_use}, {MREF[rb]}", t_shift, [t_use, MREF[rb]])
            for c in range(2):
                e.valu(f"v_mul_f32 {LSUM[rb][c]}, {t_alpha}, {LSUM[rb][c]}", LSUM[rb][c], [t_alpha, LSUM[rb][c]])
            # O[rb] *= alpha, in groups of len(scratch)
            regs = [O(rb, dt, i) for dt in range(4) for i in range(16)]
            g = len(scratch)
            for k in range(0, len(regs), g):
                grp = regs[k:k + g]
                for a_, v_ in zip(grp, scratch):
                    e.valu(f"v_accvgpr_read_b32 {v_}, {a_}", v_, [a_], kind="accr")
                for a_, v_ in zip(grp, scratch):
                    e.valu(f"v_mul_f32 {v_}, {t_alpha}, {v_}", v_, [t_alpha, v_])
                for a_, v_ in zip(grp, scratch):
                    e.valu(f"v_accvgpr_write_b32 {a_}, {v_}", a_, [v_], kind="accw")
            for t in range(2):
                for i in range(16):
                    r = S(st, rb, t, i)
                    e.valu(f"v_sub_f32 {r}, {r}, {t_shift}", r, [r, t_shift])
            e.valu(f"v_mov_b32 {MRUN[rb]}, {t_new}", MRUN[rb], [t_new])
            e.valu(f"v_mov_b32 {MREF[rb]}, {t_use}", MREF[rb], [t_use])
            e.valu(f"v_sub_f32 {THR[rb]}, {t_new}, {t_use}", THR[rb], [t_new, t_use])
            e.valu(f"v_add_f32_e32 {THR[rb]}, 0x41000000, {THR[rb]}", THR[rb], [THR[rb]])
            e.valu(f"v_sub_f32 {INIT(rb, 0)}, 0, {t_use}", INIT(rb, 0), [t_use])
            for j in range(1, 16):
                e.valu(f"v_mov_b32 {INIT(rb, j)}, {INIT(rb, 0)}", INIT(rb, j), [INIT(rb, 0)])

    def vote_and_rescale(self, st, tag):
        """One wave vote: any row of either block whose max outgrew its threshold -> rescale."""
        e = self.e
        e.valu(f"v_cmp_gt_f32_e64 {SVOTE}, {MX[0]}, {THR[0]}", None, [MX[0], THR[0]])
        e.valu(f"v_cmp_gt_f32_e64 {SVOTE2}, {MX[1]}, {THR[1]}", None, [MX[1], THR[1]])
        e.salu(f"s_or_b64 {SVOTE}, {SVOTE}, {SVOTE2}")
        e.raw(f"s_cbranch_scc0 .Lhp%=_{tag}_nr")
        self.rescale(st)
        e.label(f".Lhp%=_{tag}_nr")

    def barrier(self):
        e = self.e
        e.drain_lds()
        e.raw("s_waitcnt vmcnt(0)")
        e.raw("s_barrier")
        e.reset()

    # -- phases --------------------------------------------------------------------------------
    def qk_prologue(self, st):
        """S(0) = K(0) Q^T (+ INIT) into set st, fragments read LEADK ahead; no fillers."""
        e = self.e
        for m in range(LEADK):
            self.k_read(0, m)
        for m in range(16):
            if m + LEADK < 16:
                self.k_read(0, m + LEADK)
            t, ks = m // 8, m % 8
            for rb in range(2):
                d = S(st, rb, t)
                e.mfma(self.mop, d, KR(m % 4), f"%[q{rb * 8 + ks}]", INIT(rb) if ks == 0 else d)

    def max_mask_plain(self, st, masked):
        """Mask (masked tiles) and row max of set st, no MFMA cover (prologue)."""
        e = self.e
        if masked:
            for rb in range(2):
                e.valu(f"v_subrev_u32 {REL[rb]}, {SN1}, %[rel{rb}]", REL[rb], [])
        for rb in range(2):
            for t in range(2):
                if masked:
                    for i in range(16):
                        self.mask_elem(st, rb, t, i)
                for (txt, d, srcs) in self.max_ops(st, rb, t):
                    e.valu(txt, d, srcs)
        self.row_max_finish()

    def period_xy(self, par, cls, tag):
        """One period i (parity par) of class A (tile i+1 live, unmasked), B (live, masked) or C
        (no tile i+1): phase X = QK^T(i+1) MFMAs with the exponentials of tile i, phase Y = PV(i)
        MFMAs with the row sums of tile i and the mask / row max of tile i+1.  The fillers of each
        MFMA gap come from `GapScheduler` (deadline-ordered, issue-cost budget per gap)."""
        e = self.e
        cur, nxt = par, 1 - par
        kbuf, vbuf = 1 - par, par
        qk = cls in ("A", "B")
        masked = cls == "B"
        E = elem_order()
        self.descriptors()
        if masked:
            for rb in range(2):
                e.valu(f"v_subrev_u32 {REL[rb]}, {SN1}, %[rel{rb}]", REL[rb], [])
        dma = self.dma_stream(par)
        # ---------------- phase X ----------------
        n_x_exp = 56 if qk else 64
        gx = GapScheduler(32 if qk else 0)
        if qk:
            for m in range(16):
                if m + LEADK < 16:
                    gx.add("k", 4, 2 * m, 2 * m, lambda m=m: self.k_read(kbuf, m + LEADK))
        for n, el in enumerate(E[:n_x_exp]):
            gx.add("exp", 8, -1, (n * 30) // n_x_exp, lambda el=el: self.exp(cur, el))
        for n, f in enumerate(dma):
            gx.add("dma", f[0], -1, 4 * n + 3, f[1])
        cv = [(rb, kk, j) for kk in range(4 if not qk else 1) for rb in range(2) for j in range(4)]
        for n, c in enumerate(cv):
            gx.add("cvt", 4, -1, 31, lambda c=c: self.cvt(cur, *c))
        for m in range(LEADV):
            for h in range(2):
                gx.add("vr", 4, 20, 31, lambda m=m, h=h: self.v_read(vbuf, m, h))

        def x_mfma(g):
            m, rb = g >> 1, g & 1
            t, ks = m // 8, m % 8
            d = S(nxt, rb, t)
            e.mfma(self.mop, d, KR(m % 4), f"%[q{rb * 8 + ks}]", INIT(rb) if ks == 0 else d)

        if qk:
            for m in range(LEADK):
                self.k_read(kbuf, m)
        gx.run(x_mfma, pre_budget=40)
        # ---------------- phase Y ----------------
        gy = GapScheduler(32)
        for m in range(16):
            if m + LEADV < 16:
                for h in range(2):
                    gy.add("v", 4, 2 * m, 2 * m + 1, lambda m=m, h=h: self.v_read(vbuf, m + LEADV, h))
        for n, el in enumerate(E[n_x_exp:]):
            gy.add("exp", 8, -1, 4 + n, lambda el=el: self.exp(cur, el))
        if qk:
            for kk, dl in ((1, 5), (2, 13), (3, 21)):
                for rb in range(2):
                    for j in range(4):
                        gy.add(f"cvt{kk}", 4, -1, dl, lambda c=(rb, kk, j): self.cvt(cur, *c))
            for t in range(2):
                for rb in range(2):
                    if masked:
                        for i in range(16):
                            gy.add(f"mx{t}{rb}", 8, 16 * t - 1, 31,
                                   lambda rb=rb, t=t, i=i: self.mask_elem(nxt, rb, t, i))
                    for (txt, d, srcs) in self.max_ops(nxt, rb, t):
                        gy.add(f"mx{t}{rb}", 4, 16 * t - 1, 31,
                               lambda txt=txt, d=d, srcs=srcs: e.valu(txt, d, srcs))
        for n, el in enumerate(E):
            gy.add(f"add{n % 2}", 4, 0, 31, lambda el=el, c=n % 2: self.add(cur, el, c))

        def y_mfma(g):
            m, rb = g >> 1, g & 1
            kk, dt = m >> 2, m & 3
            e.mfma(self.mop, O(rb, dt), VR(m % 4), PF(rb, kk), O(rb, dt))

        gy.run(y_mfma, pre_budget=0)
        if qk:
            self.row_max_finish()
            self.vote_and_rescale(nxt, tag)
        e.salu(f"s_add_i32 {SI}, {SI}, 1")
        e.salu(f"s_add_i32 {SN1}, {SN1}, 64")
        self.barrier()

    def dma_stream(self, par):
        """The period's 8 LDS-DMA pieces as (cost, emit) items; each item issues its piece and
        already points m0 at the next one, so no piece waits on its own m0 write."""
        pieces = [("k", it) for it in range(4)] + [("v", it) for it in range(4)]

        def m0_of(w_, it):
            return par * 16384 + it * 4096 if w_ == "k" else 32768 + (1 - par) * 16384 + it * 4096

        out = []
        for n, (w_, it) in enumerate(pieces):
            def f(n=n, w_=w_, it=it):
                if n == 0:
                    self.e.salu(f"s_add_u32 m0, %[mlds], {m0_of(w_, it)}", m0=True)
                self.e.dma(f"buffer_load_dwordx4 %[off{it}], {SKD if w_ == 'k' else SVD}, 0 offen lds")
                if n + 1 < len(pieces):
                    self.e.salu(f"s_add_u32 m0, %[mlds], {m0_of(*pieces[n + 1])}", m0=True)
            out.append((16, f))
        return out

    def period_d(self, par):
        self.descriptors()
        for _, f in self.dma_stream(par):
            f()
        self.e.salu(f"s_add_i32 {SI}, {SI}, 1")
        self.e.salu(f"s_add_i32 {SN1}, {SN1}, 64")
        self.barrier()

    # -- the whole work item -------------------------------------------------------------------
    def build(self):
        e = self.e
        e.raw("s_nop 7")
        e.raw("s_nop 7")
        e.salu(f"s_mov_b32 {SM0}, m0")
        e.valu(f"v_mov_b32 {VNINF}, {NINF}", VNINF)
        for rb in range(2):
            e.valu(f"v_mov_b32 {MRUN[rb]}, {NINF}", MRUN[rb])
            e.valu(f"v_mov_b32 {THR[rb]}, {NINF}", THR[rb])
            e.valu(f"v_mov_b32 {MREF[rb]}, 0", MREF[rb])
            for c in range(2):
                e.valu(f"v_mov_b32 {LSUM[rb][c]}, 0", LSUM[rb][c])
            for j in range(16):
                e.valu(f"v_mov_b32 {INIT(rb, j)}, 0", INIT(rb, j))
        for rb in range(2):
            for dt in range(4):
                for i in range(16):
                    e.valu(f"v_accvgpr_write_b32 {O(rb, dt, i)}, 0", O(rb, dt, i), kind="accw")
        # DMA cursors: period i requests K(i + 2) and V(i + 1)
        e.salu(f"s_mov_b32 {SKP[0]}, %[klo]")
        e.salu(f"s_mov_b32 {SKP[1]}, %[khi]")
        e.salu(f"s_mov_b32 {SVP[0]}, %[vlo]")
        e.salu(f"s_mov_b32 {SVP[1]}, %[vhi]")
        e.salu(f"s_mov_b32 {SKR}, %[kbytes]")
        e.salu(f"s_mov_b32 {SVR}, %[kbytes]")
        for k in range(2):
            e.salu(f"s_add_u32 {SKP[0]}, {SKP[0]}, %[tileb]")
            e.salu(f"s_addc_u32 {SKP[1]}, {SKP[1]}, 0")
            e.salu(f"s_sub_i32 {SKR}, {SKR}, %[tileb]")
        e.salu(f"s_add_u32 {SVP[0]}, {SVP[0]}, %[tileb]")
        e.salu(f"s_addc_u32 {SVP[1]}, {SVP[1]}, 0")
        e.salu(f"s_sub_i32 {SVR}, {SVR}, %[tileb]")
        e.salu(f"s_mov_b32 {SI}, 0")
        e.salu(f"s_mov_b32 {SN1}, 0")
        # K(0), V(0), K(1) (requested before the statement) have landed
        e.raw("s_waitcnt vmcnt(0) lgkmcnt(0)")
        e.raw("s_barrier")
        e.reset()
        # ---- prologue: S(0) ----
        e.raw("s_cmp_lt_i32 %[last], 0")
        e.raw("s_cbranch_scc1 .Lhp%=_pro_end")
        self.qk_prologue(0)
        e.drain_lds()
        e.drain_mfma()  # both paths below start with every S(0) result readable
        e.raw("s_cmp_eq_u32 %[mask0], 0")
        e.raw("s_cbranch_scc1 .Lhp%=_pro_plain")
        self.max_mask_plain(0, True)
        self.rescale(0)
        e.raw("s_branch .Lhp%=_pro_end")
        e.label(".Lhp%=_pro_plain")
        self.max_mask_plain(0, False)
        self.rescale(0)
        e.label(".Lhp%=_pro_end")
        e.drain_mfma()
        e.raw("s_barrier")  # every wave is done with K(0) before K(2) lands in its buffer
        e.reset()
        e.salu(f"s_mov_b32 {SN1}, 64")
        # ---- class A: periods 0 .. na-1 (tile i+1 live and unmasked), unrolled by two ----
        e.raw(".balignl 64, 0xbf800000", 0)  # loop head on a 64-byte boundary, padded with s_nop 0
        e.label(".Lhp%=_A")
        e.raw(f"s_cmp_ge_i32 {SI}, %[na]")
        e.raw("s_cbranch_scc1 .Lhp%=_B")
        self.period_xy(0, "A", "a0")
        e.raw(f"s_cmp_ge_i32 {SI}, %[na]")
        e.raw("s_cbranch_scc1 .Lhp%=_B")
        self.period_xy(1, "A", "a1")
        e.raw("s_branch .Lhp%=_A")
        # ---- class B: periods na .. last-1 (tile i+1 masked) ----
        e.label(".Lhp%=_B")
        e.raw(f"s_cmp_ge_i32 {SI}, %[last]")
        e.raw("s_cbranch_scc1 .Lhp%=_C")
        e.raw(f"s_bitcmp1_b32 {SI}, 0")
        e.raw("s_cbranch_scc1 .Lhp%=_B1")
        self.period_xy(0, "B", "b0")
        e.raw("s_branch .Lhp%=_B")
        e.label(".Lhp%=_B1")
        self.period_xy(1, "B", "b1")
        e.raw("s_branch .Lhp%=_B")
        # ---- class C: period last (softmax + PV of the last live tile) ----
        e.label(".Lhp%=_C")
        e.raw(f"s_cmp_lg_u32 {SI}, %[last]")
        e.raw("s_cbranch_scc1 .Lhp%=_D")
        e.raw(f"s_bitcmp1_b32 {SI}, 0")
        e.raw("s_cbranch_scc1 .Lhp%=_C1")
        self.period_xy(0, "C", "c0")
        e.raw("s_branch .Lhp%=_D")
        e.label(".Lhp%=_C1")
        self.period_xy(1, "C", "c1")
        # ---- class D: DMA-only periods until the workgroup's last tile ----
        e.label(".Lhp%=_D")
        e.raw(f"s_cmp_ge_i32 {SI}, %[ntiles]")
        e.raw("s_cbranch_scc1 .Lhp%=_end")
        e.raw(f"s_bitcmp1_b32 {SI}, 0")
        e.raw("s_cbranch_scc1 .Lhp%=_D1")
        self.period_d(0)
        e.raw("s_branch .Lhp%=_D")
        e.label(".Lhp%=_D1")
        self.period_d(1)
        e.raw("s_branch .Lhp%=_D")
        e.label(".Lhp%=_end")
        e.raw("s_waitcnt vmcnt(0) lgkmcnt(0)")
        for rb in range(2):
            e.valu(f"v_mov_b32 %[mo{rb}], {MRUN[rb]}", None, [MRUN[rb]])
            e.valu(f"v_add_f32 %[lo{rb}], {LSUM[rb][0]}, {LSUM[rb][1]}", None, LSUM[rb])
        e.salu(f"s_mov_b32 m0, {SM0}")
        e.raw("s_nop 15")
        e.raw("s_nop 15")
        return e.out


def _asm_body(lines):
    return "\n".join(f'      "{l}\\n"' for l in lines)


def gen_fwd_function(bf16, causal):
    g = FwdGen(bf16, causal)
    lines = g.build()
    name = f"fwd_hp_main_{'bf16' if bf16 else 'f16'}_{'causal' if causal else 'full'}"
    clob = [f'"v{i}"' for i in range(N_VGPR)] + [f'"a{i}"' for i in AGPR_CLOBBER] + \
           [f'"s{i}"' for i in SGPR_CLOBBER] + ['"vcc"', '"scc"', '"memory"']
    qops = ", ".join(f'[q{i}] "a"(q[{i}])' for i in range(16))
    src = f"""// hand-placed main loop ({'bf16' if bf16 else 'fp16'}, {'causal' if causal else 'non-causal'}): {len(lines)} lines, {g.e.n_mfma} MFMAs
FA2_DEV void {name}(const u32x4 (&q)[16], const FwdHpArgs& a, float (&m_out)[2], float (&l_out)[2]) {{
  asm volatile(
{_asm_body(lines)}
      : [mo0] "=&v"(m_out[0]), [mo1] "=&v"(m_out[1]), [lo0] "=&v"(l_out[0]), [lo1] "=&v"(l_out[1])
      : {qops},
        [kb0] "v"(a.kb0), [kb1] "v"(a.kb1), [va] "v"(a.va), [vb] "v"(a.vb),
        [off0] "v"(a.off[0]), [off1] "v"(a.off[1]), [off2] "v"(a.off[2]), [off3] "v"(a.off[3]),
        [rel0] "v"(a.rel[0]), [rel1] "v"(a.rel[1]),
        [na] "s"(a.na), [last] "s"(a.last), [ntiles] "s"(a.ntiles), [mask0] "s"(a.mask0),
        [tileb] "s"(a.tileb), [kbytes] "s"(a.kbytes), [mlds] "s"(a.mlds),
        [klo] "s"(a.klo), [khi] "s"(a.khi), [vlo] "s"(a.vlo), [vhi] "s"(a.vhi)
      : {", ".join(clob)});
}}
"""
    return src


def gen_read_o():
    parts = ["// O^T accumulators a[0:127] -> registers (after the main statement's final drain)",
             "FA2_DEV void fwd_hp_read_o(f32x16 (&o)[2][4]) {"]
    for rb in range(2):
        for dt in range(4):
            base = (rb * 4 + dt) * 16
            outs = ", ".join(f'"=v"(o[{rb}][{dt}][{i}])' for i in range(16))
            body = "".join(f"v_accvgpr_read_b32 %{i}, a{base + i}\\n" for i in range(16))
            parts.append(f'  asm volatile("{body}" : {outs});')
    parts.append("}")
    return "\n".join(parts) + "\n"


def write_headers():
    os.makedirs(GEN, exist_ok=True)
    out = ["// generated by fa2_triton_amd/hp_gen.py -- do not edit", "#pragma once", "", "namespace fa2 {", ""]
    for bf16 in (True, False):
        for causal in (True, False):
            out.append(gen_fwd_function(bf16, causal))
    out.append(gen_read_o())
    out.append("}  // namespace fa2\n")
    text = "\n".join(out)
    path = os.path.join(GEN, "fwd_hp_body.h")
    if not os.path.exists(path) or open(path).read() != text:
        with open(path, "w") as f:
            f.write(text)
    return path


if __name__ == "__main__":
    print(write_headers())
