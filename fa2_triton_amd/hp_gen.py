"""Generator of the hand-placed CDNA4 (gfx950) instruction streams of the D = 128 kernels.

The hot loops of `fwd_hp_kernel`, `dq_hp_kernel` and `dkdv_hp_kernel` (csrc/*_hp_kernel.h) are
not compiler-scheduled: this module writes each as one inline-asm statement per (dtype, causal,
dropout) variant into csrc/gen/*_hp_body.h (build.py calls `write_headers()` before compiling).
Every MFMA, exponential, LDS read, LDS-DMA piece and wait is placed by the tables below, in the
spirit of cdna_hip_programming.md "4-wave, one-wave-per-SIMD, persistent structure": each
32-cycle MFMA gap carries a planned set of single-issue fillers (issue costs summed per gap),
reads are counted (`s_waitcnt lgkmcnt(N)` computed from the exact LDS issue order), and every
register hazard the hardware does not interlock (MFMA result -> vector read, vector write -> MFMA
operand, transcendental -> use, permlane source) is padded by the `Emitter` from a register-state
model, so the schedule tables only decide the ORDER.

Forward algorithm (same as the reference's compute_row_block, /root/reference/src/forward/
compute_row_blocks.py:38-103, and fwd_pipe_kernel): per 64-key tile, S^T = K Q^T (swapped so the
softmax row is one lane pair), online softmax in base 2 with defer-max (running max moved only
when a row grows by more than 8), O^T += V^T P^T.  Differences of arrangement only:
  * the scale is applied in fp32, one fma per score: z = s (scale log2 e) - m_ref, as the
    reference scales qk in fp32 (a pre-scaled-Q variant, whose LSE error exceeds the tests'
    tolerance, exists only in FA2_HP_DEV development builds: `exact=False`);
  * the row sums of P are added in the PV phase (where the VALU has room), the exponentials of a
    tile ride on the next tile's QK^T MFMAs.
The dQ (DqGen) and dK / dV (DkdvGen) streams are described at their classes.
"""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
GEN = os.path.join(HERE, "csrc", "gen")
# development timing ablations (wrong outputs; never set for a shipped build): FA2_HPGEN_ABL=a,b
ABL = set(filter(None, os.environ.get("FA2_HPGEN_ABL", "").split(",")))

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

    MFMA_RESULT = 14   # MFMA writes r  -> any non-chain access of r (8-pass XDL: 12, +2 margin)
    TO_MFMA = 3        # VALU / accvgpr_write writes r -> MFMA reads r
    TRANS_USE = 2      # v_exp writes r -> vector use
    TO_PERM = 3        # VALU writes r -> v_permlane32_swap reads r
    MFMA_READ_WAR = 2  # MFMA reads r (A/B) -> a vector instruction writes r (LDS returns land later)
    MFMA_C_WAR = 18    # MFMA reads r as C -> something writes r
    M0_DMA = 2         # s_* writes m0 -> LDS-DMA

    def __init__(self):
        self.drop = None   # development timing ablations: instructions matching it are not emitted
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

    def _window(self, kind):
        return {"mfma": self.MFMA_RESULT, "trans": self.TRANS_USE, "m0": self.M0_DMA}.get(
            kind, max(self.TO_MFMA, self.TO_PERM))

    def close_windows(self):
        """Pad until no tracked hazard window is open."""
        need = 0
        for w, k in self.wr.values():
            need = max(need, self._window(k) - (self.ws - w))
        for w in self.rd_ab.values():
            need = max(need, self.MFMA_READ_WAR - (self.ws - w))
        for w in self.rd_c.values():
            need = max(need, self.MFMA_C_WAR - (self.ws - w))
        self._pad(need)

    def snapshot(self):
        """Hazard state relative to the current position (a block boundary without a barrier)."""
        assert not self.ds, "LDS reads pending across a block boundary"
        return ({r: (self.ws - w, k) for r, (w, k) in self.wr.items()},
                {r: self.ws - w for r, w in self.rd_ab.items()},
                {r: self.ws - w for r, w in self.rd_c.items()})

    def restore(self, snaps):
        """Start a block that may follow any of the blocks whose end states are snaps: per
        register the most restrictive of them (no barrier in between)."""
        wr, ab, c = {}, {}, {}
        for swr, sab, sc in snaps:
            for r, (rel, k) in swr.items():
                rem = self._window(k) - rel
                if rem > 0 and (r not in wr or rem > wr[r][2]):
                    wr[r] = (rel, k, rem)
            for src, dst in ((sab, ab), (sc, c)):
                for r, rel in src.items():
                    dst[r] = min(rel, dst.get(r, rel))
        self.ds = []
        self.wr = {r: (self.ws - rel, k) for r, (rel, k, _) in wr.items()}
        self.rd_ab = {r: self.ws - rel for r, rel in ab.items()}
        self.rd_c = {r: self.ws - rel for r, rel in c.items()}

    def _need_lgkm(self, regs):
        hit = -1
        for j, dst in enumerate(self.ds):
            if dst & regs:
                hit = j
        if hit >= 0:
            n = len(self.ds) - 1 - hit
            # the counter holds at most 15: waiting for <= 15 outstanding covers every older read
            # (LDS reads complete in order)
            self._line(f"s_waitcnt lgkmcnt({min(n, 15)})")
            self.ds = self.ds[hit + 1:] if n <= 15 else self.ds[-15:]

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
            if r in self.rd_ab and kind != "ds":
                need = max(need, self.MFMA_READ_WAR - (self.ws - self.rd_ab[r]))
            # (an MFMA writing a register an earlier MFMA read as C: ordered by the in-order
            # matrix pipe, which reads C before any later MFMA's result lands)
            if r in self.rd_c and kind != "mfma":
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
        if self.drop and self.drop.search(text):
            return
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
        if self.drop and self.drop.search(text):
            return
        wr = set(_regs(dst))
        self._need_lgkm(wr)
        self._hazards("ds", set(_regs(addr)) if addr else set(), wr)
        self._line(text)
        self.ds.append(wr)

    def salu(self, text, m0=False):
        if self.drop and self.drop.search(text) and not m0:
            return
        self._line(text)
        if m0:
            self.wr["m0"] = (self.ws, "m0")

    def dma(self, text):
        if self.drop and self.drop.search(text):
            return
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
# dropout statement (exact scale only, where INIT(rb, 1..15) are unused): keep words W[set][rb][t]
# of the lane's row (set = tile parity; t = 32-key half) in v[177:184], and per row block the byte
# masks MC[rb][c] (byte n = 0xFF iff element (i & 3 = c, i >> 2 = n) is kept) in v[161:168];
# s[92:95] the keep-mask descriptor, s96 the byte offset of the next tile's words
FW_MD = "s[92:95]"
FW_MT = "s96"
FW_SEL = "s97"              # v_perm_b32 selector of the byte masks (mask_prep_items)
FW_TMP = ["v169", "v170"]   # per row block: the S0 source of that v_perm_b32


def FW_W(s, rb, t):
    return f"v{177 + 4 * s + 2 * rb + t}"


def FW_MC(rb, c):
    return f"v{161 + 4 * rb + c}"


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
SPAR = "s66"      # buffer parity of the current period: (i + boff) & 1
SGPR_CLOBBER = list(range(64, 92))
N_NEXT = 12 + 16  # vector-memory ops of the next-unit requests (3 tiles x 4 pieces, 16 Q loads)

LEADK = 3  # K fragments in flight ahead of their MFMAs
LEADV = 3
# round 6 experiment, off by default (FA2_HPGEN_ABL=fw_sd4 / fw_sd6): the last FW_SD PV MFMAs of a
# class A / B period run at the start of the next period, to cover the LDS latency of its first K
# fragments.  Same-box A/B (profiles/r06d_ab_fwd_schedules_*.txt): 1 % slower -- the apparent
# start-of-period latency in the stamp build was the stamp's own s_memtime wait
FW_SD = 4 if "fw_sd4" in ABL else (6 if "fw_sd6" in ABL else 0)


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

    def __init__(self, n, lds_cap=None):
        """lds_cap: at most this much LDS read weight per gap (items added with lds = their weight,
        e.g. 2 per 1 KiB ds_read_b128, 1 per 512 B ds_read_b64_tr_b16), unless at their
        deadline: the four waves of a CU share 256 B/clk of LDS reads, and a burst of reads
        queues behind itself (and a wave stalls at issue with 15 LDS operations outstanding)."""
        self.n = n
        self.items = []
        self.lds_cap = lds_cap

    def add(self, stream, cost, release, deadline, emit, lds=False):
        self.items.append(dict(stream=stream, cost=cost, rel=release, dl=deadline, emit=emit, seq=len(self.items),
                               lds=lds))

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
            nl = 0
            cap = self.lds_cap
            while True:
                el = [it for it in heads()
                      if it["rel"] <= g and not (cap is not None and it["lds"] and nl + it["lds"] > cap and it["dl"] > g)]
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
                nl += it["lds"] or 0

        fill(-1, pre_budget)
        for g in range(self.n):
            mfma(g)
            fill(g, self.BUDGET)
        while pending:  # no MFMA left to cover them
            it = heads()[0]
            pending.remove(it)
            it["emit"]()


class FwdGen:
    """exact=True: Q enters unscaled and every score gets z = s (scale log2 e) - m_ref in fp32
    (one v_fma_f32, in the PV phase beside the row max), as the reference scales qk in fp32.
    exact=False: Q pre-scaled by scale log2 e and rounded to the input dtype, the S chain seeded
    with -m_ref, so the chain yields z directly (no per-score VALU; costs one extra rounding of
    the scores, ~2^-9 relative in bf16)."""

    def __init__(self, bf16, causal, exact=True, stamp=False, dt=128, dropout=False):
        self.bf16, self.causal, self.exact, self.stamp = bf16, causal, exact, stamp
        # dropout: P is multiplied by the keep bits a dropout_mask_kernel launch wrote just before
        # (misc.hip) -- the packed P halves of dropped elements zeroed after the row sums (which
        # are of the whole P, compute_row_blocks.py:76-79); 1 / (1 - p) in the epilogue
        self.dropout = dropout
        assert not (dropout and (stamp or dt != 128 or not exact))
        # head dim: 128 (8 k-steps, 4 d-tiles) or 64 (4, 2); a 64-row K / V tile is dt / 8 KiB,
        # staged in dt / 32 LDS-DMA pieces of 4 KiB
        self.dt, self.ks, self.ndt, self.np = dt, dt // 16, dt // 32, dt // 32
        self.tile = 64 * dt * 2
        self.mop = "v_mfma_f32_32x32x16_bf16" if bf16 else "v_mfma_f32_32x32x16_f16"
        self.cvtop = "v_cvt_pk_bf16_f32" if bf16 else "v_cvt_pk_f16_f32"
        self.e = Emitter()

    def o(self, rb, dt, i=None):
        """O^T accumulators of (row block, d-tile): a[0 : 32 ndt]."""
        base = (rb * self.ndt + dt) * 16
        return rng("a", base, 16) if i is None else f"a{base + i}"

    def chain0(self, rb):
        """Initial accumulator of an S chain: 0 (exact) or INIT = -m_ref (pre-scaled Q)."""
        return "0" if self.exact else INIT(rb)

    # -- pieces ------------------------------------------------------------------------------
    def k_read(self, kbuf, m):
        """K fragment m (key half t = m // ks, k-step m % ks) of the buffer kbuf -> ring."""
        t, ks = m // self.ks, m % self.ks
        imm = kbuf * self.tile + (ks >> 1) * 4096 + 32 * t * 64
        base = "%[kb1]" if ks & 1 else "%[kb0]"
        dst = KR(m % 4)
        self.e.ds_read(f"ds_read_b128 {dst}, {base} offset:{imm}", dst)

    def v_read(self, vbuf, m, half):
        """Half `half` of V^T fragment m (kk = m // ndt, dt = m % ndt) of V buffer vbuf -> ring."""
        kk, dt = m // self.ndt, m % self.ndt
        imm = 2 * self.tile + vbuf * self.tile + dt * 4096 + 16 * kk * 64
        base = "%[vb]" if half else "%[va]"
        dst = VR(m % 4, half)
        self.e.ds_read(f"ds_read_b64_tr_b16 {dst}, {base} offset:{imm}", dst)

    def dma_piece(self, which, par, it):
        """LDS-DMA piece `it` of this wave: K(i+2) into K buffer par, V(i+1) into V buffer 1-par."""
        if which == "k":
            imm = par * self.tile + it * 4096
            desc = SKD
        else:
            imm = 2 * self.tile + (1 - par) * self.tile + it * 4096
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

    def add_pk(self, st, el):
        """LSUM[rb][0:1] += the element pair (i, i + 1) (i even), one v_pk_add_f32."""
        kk, rb, t, i = el
        r = f"v[{S(st, rb, t, i)[1:]}:{S(st, rb, t, i + 1)[1:]}]"
        l = f"v[{LSUM[rb][0][1:]}:{LSUM[rb][1][1:]}]"
        self.e.valu(f"v_pk_add_f32 {l}, {l}, {r}", l, [l, r])

    # -- dropout keep words ----------------------------------------------------------------------
    def word_load(self, s, rb, t):
        """Keep word of the lane's row in block rb, 32-key half t, of the tile at byte offset s96
        (tiled layout of fa2_amd.h: tile i at + 256 i, half t at + 128 t) -> W[s][rb][t]."""
        self.e.raw(f"buffer_load_dword {FW_W(s, rb, t)}, %[mvo{rb}], {FW_MD}, {FW_MT} offen offset:{128 * t}")

    def word_load_items(self, s):
        """The next tile's four words -> set s (issue cost 8 each), then s96 moves one tile on."""
        out = []
        for n, (rb, t) in enumerate((rb, t) for rb in range(2) for t in range(2)):
            def f(rb=rb, t=t, n=n):
                self.word_load(s, rb, t)
                if n == 3:
                    self.e.salu(f"s_add_u32 {FW_MT}, {FW_MT}, 256")
            out.append(f)
        return out

    def mask_prep_items(self, cur, rb, t):
        """W >>= 4 hh (this lane's 16 keys at bits (i & 3) + 8 (i >> 2)); MC[rb][c] = the byte mask
        whose byte n is 0xFF iff bit c + 8 n of W is set: v_perm_b32's sign selectors replicate
        bits 15 / 31 of either source into a byte, so with S1 = W << (15 - c) (bits c, c + 16 at
        15, 31) and S0 = W << (7 - c) (bits c + 8, c + 24 at 15, 31) the selector 0x0B090A08
        (s97) builds it in one instruction (bench_micro/sdwa_sext_test.hip pins it)."""
        e = self.e
        w_ = FW_W(cur, rb, t)
        tmp = FW_TMP[rb]
        out = [lambda: e.valu(f"v_lshrrev_b32 {w_}, %[hh4], {w_}", w_, [w_])]
        for c in range(4):
            mc = FW_MC(rb, c)
            out.append(lambda c=c, mc=mc: e.valu(f"v_lshlrev_b32 {mc}, {15 - c}, {w_}", mc, [w_]))
            out.append(lambda c=c: e.valu(f"v_lshlrev_b32 {tmp}, {7 - c}, {w_}", tmp, [w_]))
            out.append(lambda mc=mc: e.valu(f"v_perm_b32 {mc}, {tmp}, {mc}, {FW_SEL}", mc, [tmp, mc]))
        return out

    def mask_and(self, rb, kk, j, h):
        """Zero half h of the P pack PF[rb][kk][j] (element i = 8 (kk & 1) + 2 j + h) unless its keep
        bit is set: AND with the sign-extended byte i >> 2 (0x00 / 0xFF) of MC[rb][i & 3] (SDWA
        writes the low 16 bits of the result to the selected word: P's word is selected on the
        source too; a byte's sign extension keeps its low 7 bits, hence whole-byte masks)."""
        i = 8 * (kk & 1) + 2 * j + h
        pp, mc = PF(rb, kk, j), FW_MC(rb, i & 3)
        self.e.valu(f"v_and_b32_sdwa {pp}, sext({mc}), {pp} dst_sel:WORD_{h} dst_unused:UNUSED_PRESERVE "
                    f"src0_sel:BYTE_{i >> 2} src1_sel:WORD_{h}", pp, [mc, pp])

    def mask_and_items(self, rb, kk):
        return [lambda j=j, h=h: self.mask_and(rb, kk, j, h) for j in range(4) for h in range(2)]

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

    def fma_z(self, st, rb, t, i):
        """exact: z = s (scale log2 e) - m_ref in place (-m_ref kept in INIT(rb, 0))."""
        r = S(st, rb, t, i)
        self.e.valu(f"v_fma_f32 {r}, {r}, %[uz], {INIT(rb, 0)}", r, [r, INIT(rb, 0)])

    def max_ops_z(self, st, rb, t):
        """The row-max chain of (rb, t); in exact mode each value's fma right after the max op
        that read it."""
        out = []
        ops = self.max_ops(st, rb, t)
        covered = [[0, 1, 2]] + [[k, k + 1] for k in range(3, 15, 2)] + [[15]]
        for op, els in zip(ops, covered):
            out.append(("max",) + op)
            if self.exact:
                for i in els:
                    out.append(("fma", rb, t, i))
        return out

    def row_max_finish(self):
        """mx[rb] = max over the lane pair of max(MAH[rb][0], MAH[rb][1]) (exact: converted to the
        exponent-argument domain, mx s scale log2 e - m_ref)."""
        e = self.e
        for rb in range(2):
            e.valu(f"v_max_f32 {MX[rb]}, {MAH[rb][0]}, {MAH[rb][1]}", MX[rb], MAH[rb])
            e.valu(f"v_mov_b32 {TMP[rb]}, {MX[rb]}", TMP[rb], [MX[rb]])
        for rb in range(2):
            e.valu(f"v_permlane32_swap_b32 {MX[rb]}, {TMP[rb]}", [MX[rb], TMP[rb]], [MX[rb], TMP[rb]], kind="perm")
        for rb in range(2):
            e.valu(f"v_max_f32 {MX[rb]}, {MX[rb]}, {TMP[rb]}", MX[rb], [MX[rb], TMP[rb]])
        if self.exact:
            for rb in range(2):
                e.valu(f"v_fma_f32 {MX[rb]}, {MX[rb]}, %[uz], {INIT(rb, 0)}", MX[rb], [MX[rb], INIT(rb, 0)])

    def rescale(self, st, first=False):
        """Defer-max rescale: for each row block, m_new = max(m_run, mx + m_ref), m_use = m_new or
        0 when -inf; O, l *= exp2(m_run - m_use); z of set st -= m_use - m_ref; INIT = -m_use.
        first: the unit's first tile (O and l are still zero: nothing to scale)."""
        e = self.e
        t_new, t_use, t_alpha, t_shift = TMP[0], TMP[1], TMP[2], TMP[3]
        # free during a rescale: the row-max chains and the mask limits (MX is still read)
        scratch = [TMP[4], MAH[0][0], MAH[0][1], MAH[1][0], MAH[1][1], REL[0], REL[1]]
        for rb in range(2):
            e.valu(f"v_add_f32 {t_new}, {MX[rb]}, {MREF[rb]}", t_new, [MX[rb], MREF[rb]])
            e.valu(f"v_max_f32 {t_new}, {MRUN[rb]}, {t_new}", t_new, [MRUN[rb], t_new])
            e.valu(f"v_cmp_eq_f32_e32 vcc, {VNINF}, {t_new}", None, [VNINF, t_new])
            e.valu(f"v_cndmask_b32_e64 {t_use}, {t_new}, 0, vcc", t_use, [t_new])
            e.valu(f"v_sub_f32 {t_shift}, {t_use}, {MREF[rb]}", t_shift, [t_use, MREF[rb]])
            if not first:
                e.valu(f"v_sub_f32 {t_alpha}, {MRUN[rb]}, {t_use}", t_alpha, [MRUN[rb], t_use])
                e.valu(f"v_exp_f32 {t_alpha}, {t_alpha}", t_alpha, [t_alpha], kind="trans")
                for c in range(2):
                    e.valu(f"v_mul_f32 {LSUM[rb][c]}, {t_alpha}, {LSUM[rb][c]}", LSUM[rb][c], [t_alpha, LSUM[rb][c]])
            # O[rb] *= alpha, in groups of len(scratch)
            regs = [] if first else [self.o(rb, dt, i) for dt in range(self.ndt) for i in range(16)]
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
            if not self.exact:
                for j in range(1, 16):
                    e.valu(f"v_mov_b32 {INIT(rb, j)}, {INIT(rb, 0)}", INIT(rb, j), [INIT(rb, 0)])

    def vote_and_rescale(self, st, tag, sd=0):
        """One wave vote: any row of either block whose max outgrew its threshold -> rescale.
        sd > 0: the period's last sd PV MFMAs are deferred to the next period; a rescale runs
        them first (O must hold all of P(i) before it is scaled) and zeroes their P operands, so
        the deferred copies at the next period's start add zeros."""
        e = self.e
        e.valu(f"v_cmp_gt_f32_e64 {SVOTE}, {MX[0]}, {THR[0]}", None, [MX[0], THR[0]])
        e.valu(f"v_cmp_gt_f32_e64 {SVOTE2}, {MX[1]}, {THR[1]}", None, [MX[1], THR[1]])
        e.salu(f"s_or_b64 {SVOTE}, {SVOTE}, {SVOTE2}")
        e.raw(f"s_cbranch_scc0 .Lhp%=_{tag}_nr")
        if sd:
            self.deferred_pv(sd)
            e.drain_mfma()
        self.rescale(st)
        if sd:
            self.zero_deferred_p(sd)
        e.label(f".Lhp%=_{tag}_nr")

    def deferred_pv(self, sd, only=None):
        """The last sd PV MFMAs of a period (O^T[rb][dt] += V^T(m) P(rb, kk = 3)), run at the start of
        the next one: their operands (V^T fragments in ring slots m % 4, packs PF(rb, 3)) stay in
        registers across the barrier.  only = i: just the i-th of them."""
        e = self.e
        ny = 8 * self.ndt
        for n, g in enumerate(range(ny - sd, ny)):
            if only is not None and n != only:
                continue
            m, rb = g >> 1, g & 1
            kk, dt = m // self.ndt, m % self.ndt
            e.mfma(self.mop, self.o(rb, dt), VR(m % 4), PF(rb, kk), self.o(rb, dt))

    def zero_deferred_p(self, sd):
        """Zero the P packs the deferred MFMAs read (and, for a unit's first period, make their
        V^T ring slots finite: uninitialised accumulation registers could hold NaN patterns)."""
        e = self.e
        ny = 8 * self.ndt
        kks = sorted({((g >> 1) // self.ndt) for g in range(ny - sd, ny)})
        for rb in range(2):
            for kk in kks:
                for j in range(4):
                    e.valu(f"v_mov_b32 {PF(rb, kk, j)}, 0", PF(rb, kk, j))

    # -- s_memtime stamps (FA2_HP_STAMPS development builds only) ---------------------------------
    # per period: s[96:97] = its start (after the previous barrier), s[92:93] = the start of phase
    # Y (PV), s[94:95] = its end before the period-end waits; sums: s98 = phase X cycles, s99 =
    # phase Y + tail, %[st2] = prologue wait + every period-end wait and barrier
    def stamp_end_pre(self):
        e = self.e
        e.raw("s_memtime s[94:95]")
        e.drain_lds()
        e.raw("s_waitcnt lgkmcnt(0)")
        e.raw("s_sub_u32 s93, s94, s92")
        e.raw("s_add_u32 s99, s99, s93")
        e.raw("s_sub_u32 s92, s92, s96")
        e.raw("s_add_u32 s98, s98, s92")

    def stamp_end_post(self):
        e = self.e
        e.raw("s_memtime s[96:97]")
        e.raw("s_waitcnt lgkmcnt(0)")
        e.raw("s_sub_u32 s92, s96, s94")
        e.raw("s_add_u32 %[st2], %[st2], s92")

    def barrier(self):
        e = self.e
        if self.stamp:
            self.stamp_end_pre()
        e.drain_lds()
        e.raw("s_waitcnt vmcnt(0)")
        e.raw("s_barrier")
        if self.stamp:
            self.stamp_end_post()
        e.reset()

    # -- phases --------------------------------------------------------------------------------
    def qk_prologue(self, st):
        """S(0) = K(0) Q^T (+ INIT) into set st (K(0) in K buffer st), fragments read LEADK ahead;
        no fillers."""
        e = self.e
        nk = 2 * self.ks
        for m in range(LEADK):
            self.k_read(st, m)
        for m in range(nk):
            if m + LEADK < nk:
                self.k_read(st, m + LEADK)
            t, ks = m // self.ks, m % self.ks
            for rb in range(2):
                d = S(st, rb, t)
                e.mfma(self.mop, d, KR(m % 4), f"%[q{rb * self.ks + ks}]", self.chain0(rb) if ks == 0 else d)

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
                for op in self.max_ops_z(st, rb, t):
                    if op[0] == "max":
                        e.valu(op[1], op[2], op[3])
                    else:
                        self.fma_z(st, *op[1:])
        self.row_max_finish()

    def period_end(self, final):
        e = self.e
        e.salu(f"s_add_i32 {SI}, {SI}, 1")
        e.salu(f"s_add_i32 {SN1}, {SN1}, 64")
        e.salu(f"s_xor_b32 {SPAR}, {SPAR}, 1")
        if final:
            if self.stamp:
                self.stamp_end_pre()
            # the next unit's loads stay in flight across the epilogue (its statement waits)
            e.drain_lds()
            e.raw(f"s_waitcnt vmcnt({3 * self.np + 2 * self.ks})")
            e.raw("s_barrier")
            if self.stamp:
                self.stamp_end_post()
            e.reset()
        else:
            self.barrier()

    def next_unit_items(self, par):
        """The final period's requests: the NEXT unit's K(0) -> K buffer 1-par, V(0) -> V buffer
        1-par, K(1) -> K buffer par (all free in the final period), and its Q fragments straight
        into the Q accumulation registers (%[q*], read-write operands); N_NEXT vector-memory ops.
        Without a next unit the descriptors have range 0 (no memory access)."""
        e = self.e
        pieces = [(1 - par, "k0"), (1 - par, "v0"), (par, "k1")]

        def lds_of(buf, what, it):
            return (2 * self.tile if what == "v0" else 0) + buf * self.tile + it * 4096

        seq = [(buf, what, it) for buf, what in pieces for it in range(self.np)]
        out = []

        def desc(what):
            # s[68:71] next K tile 0 / 1, s[72:75] next V tile 0
            d = 72 if what == "v0" else 68
            return f"s[{d}:{d + 3}]"

        def build_desc():
            e.salu("s_mov_b32 s68, %[nklo]")
            e.salu("s_and_b32 s69, %[nkhi], 0xffff")
            e.salu("s_mov_b32 s70, %[nkbytes]")
            e.salu("s_mov_b32 s71, 0x20000")
            e.salu("s_mov_b32 s72, %[nvlo]")
            e.salu("s_and_b32 s73, %[nvhi], 0xffff")
            e.salu("s_mov_b32 s74, %[nkbytes]")
            e.salu("s_mov_b32 s75, 0x20000")
        out.append((8, build_desc))
        for n, (buf, what, it) in enumerate(seq):
            def f(n=n, buf=buf, what=what, it=it):
                if n == 0:
                    e.salu(f"s_add_u32 m0, %[mlds], {lds_of(buf, what, it)}", m0=True)
                if n == 2 * self.np:  # tile 1 of K: one tile further, range one tile shorter
                    e.salu("s_add_u32 s68, s68, %[tileb]")
                    e.salu("s_addc_u32 s69, s69, 0")
                    e.salu("s_sub_i32 s70, s70, %[tileb]")
                    e.salu("s_max_i32 s70, s70, 0")
                e.dma(f"buffer_load_dwordx4 %[off{it}], {desc(what)}, 0 offen lds")
                if n + 1 < len(seq):
                    e.salu(f"s_add_u32 m0, %[mlds], {lds_of(*seq[n + 1])}", m0=True)
            out.append((16, f))

        def qdesc():
            e.salu("s_mov_b32 s72, %[nqlo]")
            e.salu("s_and_b32 s73, %[nqhi], 0xffff")
            e.salu("s_mov_b32 s74, %[nqbytes]")
            e.salu("s_mov_b32 s75, 0x20000")
        out.append((8, qdesc))
        for rb in range(2):
            for ks in range(self.ks):
                def f(rb=rb, ks=ks):
                    e.raw(f"buffer_load_dwordx4 %[q{rb * self.ks + ks}], %[nqo{rb}], s[72:75], 0 offen offset:{32 * ks}")
                out.append((16, f))
        return out

    def period_xy(self, par, cls, tag, final=False):
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
        # development timing ablations of the steady-state (class A) period: FA2_HPGEN_ABL=fw_*
        # (wrong outputs; cycles only, read with the stamp build)
        drops = {"fw_nodma": r"^buffer_load|^s_add_u32 m0", "fw_noexp": r"^v_exp",
                 "fw_novalu": r"^v_(?!mfma)", "fw_nolds": r"^ds_read", "fw_nosalu": r"^s_(?!waitcnt|barrier|cbranch|nop|branch)"}
        pat = "|".join(v for k, v in drops.items() if k in ABL) if cls == "A" else ""
        e.drop = re.compile(pat) if pat else None
        if qk and self.dt == 128 and "fw_r5" not in ABL:
            # round 6: the balanced period (period_xy_bal)
            self.period_xy_bal(par, masked, tag, final, E)
            e.drop = None
            self.period_end(final)
            return
        if self.dt == 128 and FW_SD and "fw_r5" not in ABL:
            # class C follows a class A / B period (or a unit's prologue, which zeroed their
            # operands): its deferred PV MFMAs first
            self.deferred_pv(FW_SD)
        if final:
            dma = self.next_unit_items(par)
        else:
            self.descriptors()
            dma = self.dma_stream(par)
        if masked:
            for rb in range(2):
                e.valu(f"v_subrev_u32 {REL[rb]}, {SN1}, %[rel{rb}]", REL[rb], [])
        # ---------------- phase X ----------------
        nk = 2 * self.ks        # K fragments per tile (two MFMAs each)
        nx = 2 * nk             # phase X MFMAs (32 at D = 128)
        # exponentials of tile i in phase X: all but (part of) the last 16-key group, whose packs
        # come last in phase Y (D = 64: 48, the kk = 3 group in Y)
        n_x_exp = (56 if self.dt == 128 else 48) if qk else 64
        gx = GapScheduler(nx if qk else 0)
        if qk:
            for m in range(nk):
                if m + LEADK < nk:
                    gx.add("k", 4, 2 * m, 2 * m, lambda m=m: self.k_read(kbuf, m + LEADK))
        x_dl = [(n * (nx - 2)) // n_x_exp for n in range(n_x_exp)]
        for n, el in enumerate(E[:n_x_exp]):
            gx.add("exp", 8, -1, x_dl[n], lambda el=el: self.exp(cur, el))
        for n, f in enumerate(dma):
            gx.add("dma", f[0], -1, min(nx - 1, (4 * n + 3) * nx // 32), f[1])
        # a pack reads the exponentials of E[16 kk + 8 rb + 2 j], + 1 (elem_order); D = 64 orders
        # it after them explicitly (streams order only themselves: with a crowded gap a cheaper
        # item could otherwise run ahead of an exponential of another stream)
        order = self.dt == 64

        def after(idx, dls):
            return max(dls[i] for i in idx) + 1 if order else -1
        cv = [(rb, kk, j) for kk in range(4 if not qk else 1) for rb in range(2) for j in range(4)]
        for n, c in enumerate(cv):
            rb_, kk_, j_ = c
            idx = [16 * kk_ + 8 * rb_ + 2 * j_, 16 * kk_ + 8 * rb_ + 2 * j_ + 1]
            gx.add("cvt", 4, min(nx - 1, after(idx, x_dl)), nx - 1, lambda c=c: self.cvt(cur, *c))
        if self.dropout:
            # (class C only at D = 128, where A / B take period_xy_bal: phase X has no MFMA, so its
            # items run in list order after the first gap's -- released past it -- every pack first)
            assert not qk
            for rb in range(2):
                for t in range(2):
                    for f in self.mask_prep_items(cur, rb, t):
                        gx.add("dm", 4, 0, nx - 1, f)
                    for kk in (2 * t, 2 * t + 1):
                        for f in self.mask_and_items(rb, kk):
                            gx.add("dm", 4, 0, nx - 1, f)
        for m in range(LEADV):
            for h in range(2):
                gx.add("vr", 4, max(0, nx - 12), nx - 1, lambda m=m, h=h: self.v_read(vbuf, m, h))

        def x_mfma(g):
            m, rb = g >> 1, g & 1
            t, ks = m // self.ks, m % self.ks
            d = S(nxt, rb, t)
            e.mfma(self.mop, d, KR(m % 4), f"%[q{rb * self.ks + ks}]", self.chain0(rb) if ks == 0 else d)

        if qk:
            for m in range(LEADK):
                self.k_read(kbuf, m)
        gx.run(x_mfma, pre_budget=40)
        if self.stamp:
            e.raw("s_memtime s[92:93]")
        # ---------------- phase Y ----------------
        nv = 4 * self.ndt       # V^T fragments per tile (two MFMAs each)
        ny = 2 * nv             # phase Y MFMAs (32 at D = 128)
        gy = GapScheduler(ny)
        for m in range(nv):
            if m + LEADV < nv:
                for h in range(2):
                    gy.add("v", 4, 2 * m, 2 * m + 1, lambda m=m, h=h: self.v_read(vbuf, m + LEADV, h))
        n_y_exp = len(E) - n_x_exp
        y_dl = {}  # element index -> deadline of its exponential in phase Y
        for n, el in enumerate(E[n_x_exp:]):
            dl = 4 + n if self.dt == 128 else 2 + (n * 6) // max(1, n_y_exp)
            y_dl[n_x_exp + n] = dl
            gy.add("exp", 8, -1, dl, lambda el=el: self.exp(cur, el))

        def after_y(idx):
            return max([y_dl[i] for i in idx if i in y_dl] + [-2]) + 1 if order else -1
        if qk:
            # packs of P(kk) before the first PV MFMA reading them (MFMA 2 ndt kk)
            for kk in (1, 2, 3):
                dl = (5, 13, 21)[kk - 1] if self.dt == 128 else 2 * self.ndt * kk - 3
                for rb in range(2):
                    for j in range(4):
                        idx = [16 * kk + 8 * rb + 2 * j, 16 * kk + 8 * rb + 2 * j + 1]
                        gy.add(f"cvt{kk}", 4, after_y(idx), dl, lambda c=(rb, kk, j): self.cvt(cur, *c))
            for t in range(2):
                for rb in range(2):
                    if masked:
                        for i in range(16):
                            gy.add(f"mx{t}{rb}", 8, (ny // 2) * t - 1, ny - 1,
                                   lambda rb=rb, t=t, i=i: self.mask_elem(nxt, rb, t, i))
                    for op in self.max_ops_z(nxt, rb, t):
                        if op[0] == "max":
                            gy.add(f"mx{t}{rb}", 4, (ny // 2) * t - 1, ny - 1,
                                   lambda op=op: e.valu(op[1], op[2], op[3]))
                        else:
                            gy.add(f"mx{t}{rb}", 4, (ny // 2) * t - 1, ny - 1, lambda op=op: self.fma_z(nxt, *op[1:]))
        for n, el in enumerate(E):
            gy.add(f"add{n % 2}", 4, max(0, after_y([n])), ny - 1, lambda el=el, c=n % 2: self.add(cur, el, c))

        def y_mfma(g):
            m, rb = g >> 1, g & 1
            kk, dt = m // self.ndt, m % self.ndt
            e.mfma(self.mop, self.o(rb, dt), VR(m % 4), PF(rb, kk), self.o(rb, dt))

        gy.run(y_mfma, pre_budget=0)
        if qk:
            self.row_max_finish()
            self.vote_and_rescale(nxt, tag)
        e.drop = None
        self.period_end(final)

    def row_max_finish_items(self):
        """row_max_finish as a list of emit functions (scheduled into the last PV gaps)."""
        e = self.e
        out = []
        for rb in range(2):
            out.append(lambda rb=rb: e.valu(f"v_max_f32 {MX[rb]}, {MAH[rb][0]}, {MAH[rb][1]}", MX[rb], MAH[rb]))
            out.append(lambda rb=rb: e.valu(f"v_mov_b32 {TMP[rb]}, {MX[rb]}", TMP[rb], [MX[rb]]))
        for rb in range(2):
            out.append(lambda rb=rb: e.valu(f"v_permlane32_swap_b32 {MX[rb]}, {TMP[rb]}", [MX[rb], TMP[rb]],
                                            [MX[rb], TMP[rb]], kind="perm"))
        for rb in range(2):
            out.append(lambda rb=rb: e.valu(f"v_max_f32 {MX[rb]}, {MX[rb]}, {TMP[rb]}", MX[rb], [MX[rb], TMP[rb]]))
        if self.exact:
            for rb in range(2):
                out.append(lambda rb=rb: e.valu(f"v_fma_f32 {MX[rb]}, {MX[rb]}, %[uz], {INIT(rb, 0)}", MX[rb],
                                                [MX[rb], INIT(rb, 0)]))
        return out

    def period_xy_bal(self, par, masked, tag, final, E):
        """Class A / B period at D = 128 with the fillers balanced over both phases (round 6).

        The round-5 schedule put 56 of the 64 exponentials of tile i into phase X (two or three per
        MFMA gap, where one v_exp per gap hides) and left phase Y with every row sum and the whole
        mask / row max / exponent-argument pass of tile i+1 -- more than its 32 gaps hold, so ~60
        instructions ran after its last MFMA (s_memtime stamps, profiles/r06a_fwd_stamps_ablations.jsonl:
        X 1369 and Y 1400 cycles per period against 1024 of MFMAs).  Here:
          X: K fragment reads (issued first in the period, before the descriptor updates), the
             exponentials of E[0:40] (kk = 0, 1 and half of kk = 2), the packs of kk = 0 and 1, the row
             sums of kk = 0, the LDS-DMA pieces, and -- once the chains S(i+1)[rb][t = 0] are complete
             (MFMAs 14, 15) -- the t = 0 half of the mask / row max / exponent arguments of tile i+1;
          Y: the remaining 24 exponentials, the kk = 2, 3 packs, the other row sums, the t = 1 half of
             the next tile's pass, and the row-max finish in its last gaps (the vote after the last
             MFMA).
        Every cross-stream dependence is a release after the producer's deadline (a stream orders
        only itself)."""
        e = self.e
        cur, nxt = par, 1 - par
        kbuf, vbuf = 1 - par, par
        nk, nx, nv = 2 * self.ks, 4 * self.ks, 4 * self.ndt
        sd = FW_SD
        ny = 2 * nv - sd  # this period's PV MFMAs; the last sd run at the next period's start
        # the first K fragments first: their LDS latency runs under the scalar updates below
        for m in range(LEADK):
            self.k_read(kbuf, m)
        if final:
            dma = self.next_unit_items(par)
        else:
            self.descriptors()
            dma = self.dma_stream(par)
        if masked:
            for rb in range(2):
                e.valu(f"v_subrev_u32 {REL[rb]}, {SN1}, %[rel{rb}]", REL[rb], [])

        def zprep(add, t, rb, release, deadline):
            st_ = f"mx{t}{rb}"
            if masked:
                for i in range(16):
                    add(st_, 8, release, deadline, lambda rb=rb, t=t, i=i: self.mask_elem(nxt, rb, t, i))
            for op in self.max_ops_z(nxt, rb, t):
                if op[0] == "max":
                    add(st_, 4, release, deadline, lambda op=op: e.valu(op[1], op[2], op[3]))
                else:
                    add(st_, 4, release, deadline, lambda op=op: self.fma_z(nxt, *op[1:]))

        # ---------------- phase X ----------------
        # gap indices of phase X count from its first QK^T MFMA (the sd deferred PV MFMAs before it
        # are gaps -sd .. -1); GapScheduler positions are those + sd
        n_x = 40
        x_dl = {n: (n * 28) // n_x for n in range(n_x)}
        gx = GapScheduler(nx + sd)

        def gxa(stream, cost, rel, dl, f):
            gx.add(stream, cost, rel + sd if rel >= 0 else rel, dl + sd, f)
        for m in range(nk):
            if m + LEADK < nk:
                gxa("k", 4, 2 * m, 2 * m, lambda m=m: self.k_read(kbuf, m + LEADK))
        # (released one gap before the deadline: about one exponential per gap instead of a burst of
        # three, MI355X_MICROARCH.md filler rule "at most one v_exp per MFMA gap")
        for n in range(n_x):
            gxa("exp", 8, x_dl[n] - 1, x_dl[n], lambda el=E[n]: self.exp(cur, el))
        for n, f in enumerate(dma):
            gxa("dma", f[0], -1, min(nx - 1, (4 * n + 3) * nx // 32), f[1])
        # dropout: the kk = 0 packs early enough for their keep masking in phase X (X_CVT0); the
        # next tile's keep words requested at the period start
        X_CVT0 = 20
        for kk in (0, 1):
            for rb in range(2):
                for j in range(4):
                    idx = [16 * kk + 8 * rb + 2 * j, 16 * kk + 8 * rb + 2 * j + 1]
                    gxa(f"cvt{kk}", 4, max(x_dl[i] for i in idx) + 1, X_CVT0 if self.dropout and kk == 0 else nx - 1,
                        lambda c=(rb, kk, j): self.cvt(cur, *c))
        if self.dropout:
            for f in self.word_load_items(nxt):
                gxa("wl", 8, -1, 6, f)
            for rb in range(2):
                for f in self.mask_prep_items(cur, rb, 0):
                    gxa(f"dm{rb}", 4, -1, X_CVT0 - 2, f)
                for f in self.mask_and_items(rb, 0):
                    gxa(f"dm{rb}", 4, X_CVT0 + 1, nx - 1, f)
        if "fw_pk" in ABL:  # (A/B: row sums of element pairs by v_pk_add_f32, same partial sums)
            for n in range(0, 16, 2):
                gxa("add", 8, max(x_dl[n], x_dl[n + 1]) + 1, nx - 1, lambda el=E[n]: self.add_pk(cur, el))
        else:
            for n in range(16):
                gxa(f"add{n % 2}", 4, x_dl[n] + 1, nx - 1, lambda el=E[n], c=n % 2: self.add(cur, el, c))
        for m in range(LEADV):
            for h in range(2):
                gxa("vr", 4, max(0, nx - 12), nx - 1, lambda m=m, h=h: self.v_read(vbuf, m, h))
        # S(i+1)[rb][0] is complete after MFMA 14 + rb
        for rb in range(2):
            zprep(gxa, 0, rb, 17 + rb, nx - 1)

        def x_mfma(g):
            if g < sd:  # the previous period's deferred PV MFMAs (zeros after a unit start / rescale)
                self.deferred_pv(sd, only=g)
                return
            g -= sd
            m, rb = g >> 1, g & 1
            t, ks = m // self.ks, m % self.ks
            d = S(nxt, rb, t)
            e.mfma(self.mop, d, KR(m % 4), f"%[q{rb * self.ks + ks}]", self.chain0(rb) if ks == 0 else d)

        # (before the first MFMA the wave waits for its first K fragment anyway: room for fillers)
        gx.run(x_mfma, pre_budget=64)
        if self.stamp:
            e.raw("s_memtime s[92:93]")
        # ---------------- phase Y ----------------
        gy = GapScheduler(ny)
        for m in range(nv):
            if m + LEADV < nv:
                for h in range(2):
                    gy.add("v", 4, 2 * m, 2 * m + 1, lambda m=m, h=h: self.v_read(vbuf, m + LEADV, h))
        # (dropout: exponentials and packs earlier, so that the keep masking of a pack fits between
        # it and the first PV MFMA reading it, MFMA 8 kk)
        y_span = 16 if self.dropout else 20
        y_dl = {n: ((n - n_x) * y_span) // (64 - n_x) for n in range(n_x, 64)}
        for n in range(n_x, 64):
            gy.add("exp", 8, y_dl[n] - 1, y_dl[n], lambda el=E[n]: self.exp(cur, el))
        # packs of P(kk) before the first PV MFMA reading them (MFMA 8 kk; margin for VALU -> MFMA)
        y_cvt = (9, 17) if self.dropout else (13, 21)
        for kk in (2, 3):
            for rb in range(2):
                for j in range(4):
                    idx = [16 * kk + 8 * rb + 2 * j, 16 * kk + 8 * rb + 2 * j + 1]
                    rel = max([y_dl[i] for i in idx if i in y_dl] + [-2]) + 1
                    gy.add(f"cvt{kk}", 4, rel, y_cvt[kk - 2], lambda c=(rb, kk, j): self.cvt(cur, *c))
        if self.dropout:
            for rb in range(2):
                for f in self.mask_and_items(rb, 1):
                    gy.add(f"dm{rb}", 4, -1, 5, f)
                for f in self.mask_prep_items(cur, rb, 1):
                    gy.add(f"dm{rb}", 4, -1, 8, f)
                for kk in (2, 3):
                    for f in self.mask_and_items(rb, kk):
                        gy.add(f"dm{rb}", 4, y_cvt[kk - 2] + 1, 8 * kk - 2, f)
        if "fw_pk" in ABL:
            for n in range(16, 64, 2):
                rel = max(y_dl.get(n, -2), y_dl.get(n + 1, -2)) + 1
                gy.add("add", 8, rel, ny - 1, lambda el=E[n]: self.add_pk(cur, el))
        else:
            for n in range(16, 64):
                rel = y_dl[n] + 1 if n in y_dl else -1
                gy.add(f"add{n % 2}", 4, rel, ny - 1, lambda el=E[n], c=n % 2: self.add(cur, el, c))
        for rb in range(2):
            zprep(gy.add, 1, rb, -1, ny - 4)
        for f in self.row_max_finish_items():
            gy.add("rmf", 4, ny - 3, ny - 1, f)

        def y_mfma(g):
            m, rb = g >> 1, g & 1
            kk, dt = m // self.ndt, m % self.ndt
            e.mfma(self.mop, self.o(rb, dt), VR(m % 4), PF(rb, kk), self.o(rb, dt))

        gy.run(y_mfma, pre_budget=0)
        self.vote_and_rescale(nxt, tag, sd)

    def dma_stream(self, par):
        """The period's 8 LDS-DMA pieces as (cost, emit) items; each item issues its piece and
        already points m0 at the next one, so no piece waits on its own m0 write."""
        pieces = [("k", it) for it in range(self.np)] + [("v", it) for it in range(self.np)]

        def m0_of(w_, it):
            return par * self.tile + it * 4096 if w_ == "k" else 2 * self.tile + (1 - par) * self.tile + it * 4096

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

    def period_d(self, par, final=False):
        if self.stamp:
            self.e.raw("s_memtime s[92:93]")
        if final:
            items = self.next_unit_items(par)
        else:
            self.descriptors()
            items = self.dma_stream(par)
        for _, f in items:
            f()
        self.period_end(final)

    # -- one work unit (256 query rows), persistent across units --------------------------------
    def build(self):
        e = self.e
        e.raw("s_nop 7")
        e.raw("s_nop 7")
        if self.stamp:
            e.raw("s_memtime s[100:101]")
            e.raw("s_mov_b32 s98, 0")
            e.raw("s_mov_b32 s99, 0")
        e.salu(f"s_mov_b32 {SM0}, m0")
        e.valu(f"v_mov_b32 {VNINF}, {NINF}", VNINF)
        for rb in range(2):
            e.valu(f"v_mov_b32 {MRUN[rb]}, {NINF}", MRUN[rb])
            e.valu(f"v_mov_b32 {THR[rb]}, {NINF}", THR[rb])
            e.valu(f"v_mov_b32 {MREF[rb]}, 0", MREF[rb])
            for c in range(2):
                e.valu(f"v_mov_b32 {LSUM[rb][c]}, 0", LSUM[rb][c])
            for j in range(1 if self.exact else 16):
                e.valu(f"v_mov_b32 {INIT(rb, j)}, 0", INIT(rb, j))
        for rb in range(2):
            for dt in range(self.ndt):
                for i in range(16):
                    e.valu(f"v_accvgpr_write_b32 {self.o(rb, dt, i)}, 0", self.o(rb, dt, i), kind="accw")
        if self.dt == 128 and FW_SD and "fw_r5" not in ABL:
            # the first period's deferred PV MFMAs add V^T x 0: zero packs, finite V^T ring slots
            self.zero_deferred_p(FW_SD)
            ny = 8 * self.ndt
            for slot in sorted({((g >> 1) % 4) for g in range(ny - FW_SD, ny)}):
                for r in _regs(VR(slot)):
                    e.valu(f"v_accvgpr_write_b32 {r}, 0", r, kind="accw")
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
        e.salu(f"s_mov_b32 {SPAR}, %[boff]")
        if self.dropout:
            # the keep-mask descriptor; tile 0's words into both sets (its period's parity is boff)
            e.salu("s_mov_b32 s92, %[mlo]")
            e.salu("s_mov_b32 s93, %[mhi]")
            e.salu("s_mov_b32 s94, %[mbytes]")
            e.salu("s_mov_b32 s95, 0x20000")
            e.salu(f"s_mov_b32 {FW_MT}, 0")
            e.salu(f"s_mov_b32 {FW_SEL}, 0x0b090a08")
            for s_ in range(2):
                for rb in range(2):
                    for t in range(2):
                        self.word_load(s_, rb, t)
            e.salu(f"s_mov_b32 {FW_MT}, 256")
        # this unit's K(0), V(0), K(1) and Q (requested during the previous unit's final period,
        # or before the statement) have landed
        e.raw("s_waitcnt vmcnt(0) lgkmcnt(0)")
        e.raw("s_barrier")
        if self.stamp:  # prologue wait (st2 then adds every period-end wait)
            e.raw("s_memtime s[92:93]")
            e.raw("s_waitcnt lgkmcnt(0)")
            e.raw("s_sub_u32 s92, s92, s100")
            e.raw("s_mov_b32 %[st2], s92")
        e.reset()
        # ---- prologue: S(0) in set boff (K(0) in K buffer boff) ----
        e.raw("s_cmp_lt_i32 %[last], 0")
        e.raw("s_cbranch_scc1 .Lhp%=_pro_end")
        for par in (0, 1):
            e.label(f".Lhp%=_pro{par}")
            if par == 0:
                e.raw(f"s_cmp_eq_u32 {SPAR}, 1")
                e.raw("s_cbranch_scc1 .Lhp%=_pro1")
            self.qk_prologue(par)
            e.drain_lds()
            e.drain_mfma()  # both paths below start with every S(0) result readable
            e.raw("s_cmp_eq_u32 %[mask0], 0")
            e.raw(f"s_cbranch_scc1 .Lhp%=_pro{par}_plain")
            self.max_mask_plain(par, True)
            self.rescale(par, first=True)
            e.raw("s_branch .Lhp%=_pro_end")
            e.label(f".Lhp%=_pro{par}_plain")
            self.max_mask_plain(par, False)
            self.rescale(par, first=True)
            e.raw("s_branch .Lhp%=_pro_end")
        e.label(".Lhp%=_pro_end")
        e.drain_mfma()
        e.raw("s_barrier")  # every wave is done with K(0) before K(2) lands in its buffer
        if self.stamp:  # the first period starts here
            e.raw("s_memtime s[96:97]")
            e.raw("s_waitcnt lgkmcnt(0)")
        e.reset()
        e.salu(f"s_mov_b32 {SN1}, 64")
        e.salu("s_add_i32 s67, %[ntiles], -1")  # s67: index of the final period
        e.raw("s_cmp_lt_i32 s67, 0")
        e.raw("s_cbranch_scc1 .Lhp%=_noper")
        # ---- periods 0 .. ntiles-2: class by tile i+1, body by parity ----
        e.raw(".balignl 64, 0xbf800000", 0)  # loop head on a 64-byte boundary, padded with s_nop 0
        e.label(".Lhp%=_loop")
        e.raw(f"s_cmp_ge_i32 {SI}, s67")
        e.raw("s_cbranch_scc1 .Lhp%=_fin")
        e.raw(f"s_cmp_lt_i32 {SI}, %[na]")
        e.raw("s_cbranch_scc1 .Lhp%=_clsA")
        e.raw(f"s_cmp_lt_i32 {SI}, %[last]")
        e.raw("s_cbranch_scc1 .Lhp%=_clsB")
        e.raw(f"s_cmp_eq_u32 {SI}, %[last]")
        e.raw("s_cbranch_scc1 .Lhp%=_clsC")
        e.raw(f"s_cmp_eq_u32 {SPAR}, 0")
        e.raw("s_cbranch_scc1 .Lhp%=_D0")
        e.raw("s_branch .Lhp%=_D1")
        # class A runs as a chain: one compare and one (mostly not taken) branch per period
        e.label(".Lhp%=_clsA")
        e.raw(f"s_cmp_eq_u32 {SPAR}, 0")
        e.raw("s_cbranch_scc0 .Lhp%=_A1")
        e.label(".Lhp%=_A0")
        self.period_xy(0, "A", "a0")
        e.raw(f"s_cmp_ge_i32 {SI}, %[na]")
        e.raw("s_cbranch_scc1 .Lhp%=_loop")
        e.label(".Lhp%=_A1")
        self.period_xy(1, "A", "a1")
        e.raw(f"s_cmp_lt_i32 {SI}, %[na]")
        e.raw("s_cbranch_scc1 .Lhp%=_A0")
        e.raw("s_branch .Lhp%=_loop")
        for cls in ("B", "C"):
            e.label(f".Lhp%=_cls{cls}")
            e.raw(f"s_cmp_eq_u32 {SPAR}, 0")
            e.raw(f"s_cbranch_scc0 .Lhp%=_{cls}1")
            for par in (0, 1):
                e.label(f".Lhp%=_{cls}{par}")
                self.period_xy(par, cls, f"{cls.lower()}{par}")
                e.raw("s_branch .Lhp%=_loop")
        for par in (0, 1):
            e.label(f".Lhp%=_D{par}")
            self.period_d(par)
            e.raw("s_branch .Lhp%=_loop")
        # ---- the final period (i = ntiles - 1): class C or D, the next unit's requests ----
        e.label(".Lhp%=_fin")
        e.raw(f"s_cmp_eq_u32 {SI}, %[last]")
        e.raw("s_cbranch_scc0 .Lhp%=_finD")
        e.raw(f"s_cmp_eq_u32 {SPAR}, 0")
        e.raw("s_cbranch_scc0 .Lhp%=_finC1")
        for par in (0, 1):
            e.label(f".Lhp%=_finC{par}")
            self.period_xy(par, "C", f"fc{par}", final=True)
            e.raw("s_branch .Lhp%=_end")
        e.label(".Lhp%=_finD")
        e.raw(f"s_cmp_eq_u32 {SPAR}, 0")
        e.raw("s_cbranch_scc0 .Lhp%=_finD1")
        for par in (0, 1):
            e.label(f".Lhp%=_finD{par}")
            self.period_d(par, final=True)
            e.raw("s_branch .Lhp%=_end")
        # ---- no period at all: the next unit's requests right away (every buffer is free) ----
        e.label(".Lhp%=_noper")
        e.raw(f"s_cmp_eq_u32 {SPAR}, 0")
        e.raw("s_cbranch_scc1 .Lhp%=_noper1")
        for par in (0, 1):
            # parity of a virtual final period: boff ^ 1
            if par == 1:
                e.label(".Lhp%=_noper1")
            for _, f in self.next_unit_items(par):
                f()
            e.raw("s_branch .Lhp%=_end")
        e.label(".Lhp%=_end")
        e.drain_lds()
        for rb in range(2):
            e.valu(f"v_mov_b32 %[mo{rb}], {MRUN[rb]}", None, [MRUN[rb]])
            e.valu(f"v_add_f32 %[lo{rb}], {LSUM[rb][0]}, {LSUM[rb][1]}", None, LSUM[rb])
        e.salu(f"s_mov_b32 m0, {SM0}")
        if self.stamp:
            e.raw("s_memtime s[92:93]")
            e.raw("s_waitcnt lgkmcnt(0)")
            e.raw("s_sub_u32 s92, s92, s100")
            e.raw("s_mov_b32 %[st0], s98")
            e.raw("s_mov_b32 %[st1], s99")
            e.raw("s_mov_b32 %[st3], s92")
        e.raw("s_nop 15")
        e.raw("s_nop 15")
        return e.out


# ----------------------------------------------------------------------------------------------
# dK / dV (the backward's dominant kernel): dkdv_hp_kernel (csrc/dkdv_hp_kernel.h)
#
# Software-pipelined step (round 5): the step i of a wave runs, between two barriers,
#   M 0-7    the last 8 dK MFMAs of step i-1 (dK^T += Q^T dS for rows 16-31; operands read before
#            the barrier: the Q^T fragments in the row ring, the packed dS in registers), so the
#            step opens with MFMAs while its first LDS reads are in flight;
#   M 8-23   S(i+1) = Q(i+1) K^T into the other S register set (the NEXT step's scores);
#   M 24-39  dP(i) = dO(i) V^T, seeded with the -delta rows;
#   M 40-55  dV^T += dO(i)^T P(i);
#   M 56-63  dK^T += Q(i)^T dS(i), rows 0-15.
# so the exponentials of P(i) (whose S(i) the previous step computed) run beside M 0-47 and dS(i)
# beside M 41-63 (round 4 ran S(i) first and waited for it: the exponentials crowded 16 gaps).
#
# Register map of the statement:
#   v[0:63]     S[st][kb] (two sets by step parity): the next step's scores, then P = exp2(s scale
#               log2 e - LSE2) in place
#   v[64:95]    dP[kb] accumulators (start as -delta rows), then dS = P (dP - delta) in place, then
#               in place the packed dS DSP[kb][sp] (B operands of dK^T += Q^T dS)
#   v[96:111]   PP[kb][sp] packed P (B operand of dV^T += dO^T P)
#   v[112:127]  row-fragment ring, 4 slots: Q(i+1), dO(i), then the Q^T(i) fragments of rows 16-31
#               for the next step's first MFMAs
#   v[128:143]  V fragment ring (B operands of dP), 4 slots
#   v[144:159]  transposed fragment ring (dO^T, then Q^T of rows 0-15), 4 slots
#   v[160:167]  LSE2 of 8 of the lane's rows (rows of 16-row half sp, reloaded for sp = 1)
#   a[0:127]    dV^T[kb][dt], a[128:255] dK^T[kb][dt]
#   K fragments: compiler-placed "v" operands %[k0]..%[k15]
# LDS (bytes from the workgroup's base, DkLayout): a ring of nbuf = 5 step buffers -- step i
# reads buffers i and i + 1, its DMA fills buffer i + 3: Q tile of buffer b at 16384 b, dO tile at
# 16384 b + 8192 (Tile<128, 32>; buffer 4 through the "h" bases, 64 KiB up: a ds offset has 16
# bits), V rows of wave w at v0 + 16384 w (Tile<128, 64>), LSE2 / -delta rows of buffer b at
# rows + 256 b (+128).
# One barrier per TWO steps (after the odd ones): between the barriers after steps j - 2 and j
# (j odd) the steps j - 1 and j read buffers j - 1 .. j + 1 and request steps j + 2 and j + 3
# into the buffers of steps j - 3 and j - 2, which every wave finished reading before the
# barrier after step j - 2: five buffers.  At that barrier every request so far has landed
# (vmcnt(0): the odd step's own request is issued early in the step).  The S / P register set
# alternates per step, so the step bodies come in 10 phases (buffer ph % 5, set ph & 1).
# The dropout statement keeps four buffers and a barrier after every step (the "h" bases of
# buffer 4 would spill its VGPRs); FA2_HPGEN_ABL=dk_nb4 gives the plain one the same.
DK_NBUF_PLAIN = 4 if "dk_nb4" in ABL else 5
DK_NBUF_DROP = 4


class DkLayout:
    """LDS layout of one dK/dV statement variant (bytes from the workgroup's base)."""

    def __init__(self, nbuf):
        self.nbuf = nbuf
        self.ph = nbuf if nbuf % 2 == 0 else 2 * nbuf  # step phases: buffer ph % nbuf, set ph & 1
        self.halfbar = nbuf == 5
        self.v0 = 16384 * nbuf
        self.rows = self.v0 + 65536
        self.lds = self.rows + 256 * nbuf
        self.w0 = self.lds  # dropout: keep words of buffer b, wave w at w0 + 1024 b + 256 w
        self.lds_drop = self.w0 + 1024 * nbuf


DK_AHEAD = 3  # a step's DMA fills the buffer of the step DK_AHEAD later
DK_VMEM = 4  # vector-memory ops of one step's DMA after its rows (the count each step end leaves)


def DS(st, kb, i=None):
    base = 32 * st + 16 * kb
    return rng("v", base, 16) if i is None else f"v{base + i}"


def DDP(kb, i=None):
    return rng("v", 64 + 16 * kb, 16) if i is None else f"v{64 + 16 * kb + i}"


def DDSP(kb, sp, j=None):
    """Packed dS of 16-row half sp, in place over dP[kb] (as QDSP): pack j of elements 8 sp ..
    8 sp + 7 reads 2j, 2j + 1 and writes element j."""
    base = 64 + 16 * kb + 8 * sp
    return rng("v", base, 4) if j is None else f"v{base + j}"


def DPP(kb, sp, j=None):
    base = 96 + (kb * 2 + sp) * 4
    return rng("v", base, 4) if j is None else f"v{base + j}"


def DRR(slot, half=None):
    base = 112 + 4 * (slot % 4)
    return rng("v", base, 4) if half is None else rng("v", base + 2 * half, 2)


DVF_SLOTS = 5 if "dk_vf5" in ABL else 4


def DVF(n):
    return rng("v", 128 + 4 * (n % DVF_SLOTS), 4)


def DTR(slot, half=None):
    base = 144 + 4 * (slot % 4)
    return rng("v", base, 4) if half is None else rng("v", base + 2 * half, 2)


DLSE0 = 160 + (4 if "dk_vf5" in ABL else 0)


def DLSE(i):
    """LSE2 of the row of register i (rows (i & 3) + 8 (i >> 2) + 4 hh of the step's tile); the
    8 registers hold the rows of one half sp = i >> 3 at a time."""
    return f"v{DLSE0 + (i & 7)}"


DK_NVGPR = DLSE0 + 8
# dropout (the forward's saved keep words, DkdvGen(dropout=True)):
#   DKM[kb]   the lane's keep column of key block kb (bit (i & 3) + 8 (i >> 2) = register i's row)
#   DTM[kb]   temporary of key block kb: the P packs' masking, then the dS keep factors
#   -delta of row group g4 (rows 8 g4 + 4 hh ..) in V fragment ring slot g4 (the ring is free from
#   the dP MFMA that last reads a slot to the next step's first V fragment read)
DKM = [f"v{DK_NVGPR}", f"v{DK_NVGPR + 1}"]
DTM = [f"v{DK_NVGPR + 2}", f"v{DK_NVGPR + 3}"]
DK_NVGPR_DROP = DK_NVGPR + 4
D_MC = "s99"       # dropout: byte offset of the requested step's keep words from the wave's base


def _lds_hi(buf, imm, base):
    """(base operand, offset) of an LDS read at step-buffer offset imm: buffer 4 through the
    operand's "h" twin (64 KiB up)."""
    return (base[:-1] + "h]", imm - 65536) if imm >= 65536 else (base, imm)


def DDEL(g4, j=None):
    base = 128 + 4 * g4
    return rng("v", base, 4) if j is None else f"v{base + j}"



def DDV(kb, dt):
    return rng("a", (kb * 4 + dt) * 16, 16)


def DDK(kb, dt):
    return rng("a", 128 + (kb * 4 + dt) * 16, 16)


# scalar state of the dK/dV statement
D_G = "s64"        # q-head index in the group
D_IDX = "s65"      # step index within the head
D_CM = "s66"       # first query row of the current tile
# descriptors of the requested step's Q, dO, LSE2 and delta rows; their base words ARE the
# cursors (the requested tile's first byte; stride 0, and a 48-bit address leaves the high
# word's stride bits clear), word 2 the range of the step, word 3 constant
D_QD = "s[68:71]"
D_OD = "s[72:75]"
D_LD = "s[76:79]"
D_DD = "s[80:83]"
D_QP = ("s68", "s69")
D_OP = ("s72", "s73")
D_LP = ("s76", "s77")
D_DP = ("s80", "s81")
D_MD = "s[84:87]"  # dropout: keep-word descriptor (constant through the statement)
D_WL = "s88"       # dropout: LDS base of this wave's keep words in buffer 0
D_NM = "s89"       # requested step's first query row
D_LEFT = "s90"     # total steps - the requested step's index (> 0: it exists)
D_NMT = "s91"      # requested step's tile index within its head
D_M0 = "s92"
D_T = "s93"
D_EX = "s[94:95]"  # exec save of the rows DMA
D_MK = ["s[96:97]", "s[98:99]"]


class DkdvGen:
    """dK / dV: 4 waves x 64 keys (two 32-key blocks kb per wave, one wave per SIMD); per step
    (32 query rows of one q-head) 64 MFMAs: S(i+1)[kb] = Q K'^T (16), dP(i)[kb] = dO V^T (16),
    dV^T[kb] += dO^T P (16), dK^T[kb] += Q^T dS (16, 8 of them in the next step); every Q / dO /
    transposed fragment read from LDS feeds both key blocks.  Same math as the reference's dK/dV
    loop (/root/reference/src/backward/compute_dkdv.py:42-112) and dkdv_kernel."""

    def __init__(self, bf16, causal, dropout=False):
        self.bf16, self.causal, self.dropout = bf16, causal, dropout
        assert not (dropout and DVF_SLOTS != 4), "the dropout -delta rows use the V ring's 4 slots"
        self.vslots = DVF_SLOTS
        self.L = DkLayout(DK_NBUF_DROP if dropout else DK_NBUF_PLAIN)
        self.nvgpr = DK_NVGPR_DROP if dropout else DK_NVGPR
        self.mop = "v_mfma_f32_32x32x16_bf16" if bf16 else "v_mfma_f32_32x32x16_f16"
        self.cvtop = "v_cvt_pk_bf16_f32" if bf16 else "v_cvt_pk_f16_f32"
        self.e = Emitter()

    # -- pieces ----------------------------------------------------------------------------------
    def row_read(self, buf, dout, ks):
        """Row fragment ks (Q, or dO when dout) of buffer buf into ring slot ks % 4."""
        imm = buf * 16384 + (8192 if dout else 0) + (ks >> 1) * 2048
        base, imm = _lds_hi(buf, imm, "%[qb1]" if ks & 1 else "%[qb0]")
        d = DRR(ks)
        self.e.ds_read(f"ds_read_b128 {d}, {base} offset:{imm}", d)

    def v_frag(self, n):
        """V fragment n = 2 ks + kb (keys 32 kb .. of this wave, k-step ks)."""
        ks, kb = n >> 1, n & 1
        imm = (ks >> 1) * 4096 + 32 * kb * 64
        base = "%[vb1]" if ks & 1 else "%[vb0]"
        d = self.dvf(n)
        self.e.ds_read(f"ds_read_b128 {d}, {base} offset:{imm}", d)

    def tr_read(self, buf, dout, f, half, dst):
        """Half `half` of transposed fragment f (sp = f >> 2, dt = f & 3) of dO^T (dout) or Q^T of
        buffer buf into the 2 registers dst."""
        sp, dt = f >> 2, f & 3
        imm = buf * 16384 + (8192 if dout else 0) + dt * 2048 + 16 * sp * 64
        base, imm = _lds_hi(buf, imm, "%[tb]" if half else "%[ta]")
        self.e.ds_read(f"ds_read_b64_tr_b16 {dst}, {base} offset:{imm}", dst)

    def dvf(self, n):
        return rng("v", 128 + 4 * (n % self.vslots), 4)

    def init_read(self, buf, what, kb, g4):
        """LSE2 (what 0; g4 in the half's pair) rows into the LSE registers, -delta (what 1) into
        dP[kb] (the dP chain's initial accumulator): register group g4."""
        imm = buf * 256 + what * 128 + 32 * g4
        d = rng("v", DLSE0 + 4 * (g4 & 1), 4) if what == 0 else rng("v", 64 + 16 * kb + 4 * g4, 4)
        self.e.ds_read(f"ds_read_b128 {d}, %[lb] offset:{imm}", d)

    def descriptors(self, part=None):
        """The ranges of the requested step's descriptors (range 0 when none): part 0 the rows
        (D_T) and the LSE2 / delta bytes below Lq, 1 the Q and dO bytes."""
        e = self.e
        if part in (None, 0):
            e.salu(f"s_sub_u32 {D_T}, %[lq], {D_NM}")
            e.salu(f"s_cmp_gt_i32 {D_LEFT}, 0")
            e.salu(f"s_cselect_b32 {D_T}, {D_T}, 0")
            e.salu(f"s_min_u32 s78, {D_T}, 32")
            e.salu("s_lshl_b32 s78, s78, 2")
            if self.dropout:  # lsoff = sb + w0 + 256 w + 4 lane (w = 0 here): the range
                # starts there (lbs = sb + rows)
                e.salu("s_add_u32 s78, s78, %[lbs]")
                e.salu(f"s_add_u32 s78, s78, {self.L.w0 - self.L.rows}")
            e.salu("s_mov_b32 s82, s78")
        if part in (None, 1):
            orb = "%[qrb]" if self.dropout else "%[orb]"  # (dropout: one row stride)
            e.salu(f"s_mul_i32 s70, {D_T}, %[qrb]")
            e.salu(f"s_mul_i32 s74, {D_T}, {orb}")

    def advance_cursors(self, tag):
        """Cursors to the step after the requested one: one tile down, or the next head's last
        tile; one request fewer left."""
        e = self.e
        e.salu(f"s_sub_i32 {D_LEFT}, {D_LEFT}, 1")
        e.salu(f"s_add_u32 {D_NMT}, {D_NMT}, 1")
        e.salu(f"s_cmp_eq_u32 {D_NMT}, %[nmt]")
        e.raw(f"s_cbranch_scc1 .Lhp%=_{tag}_wrap")
        e.salu(f"s_sub_u32 {D_NM}, {D_NM}, 32")
        # one tile = 32 rows (D_T: free once the step's descriptors are built)
        e.salu(f"s_lshl_b32 {D_T}, %[qrb], 5")
        e.salu(f"s_sub_u32 {D_QP[0]}, {D_QP[0]}, {D_T}")
        e.salu(f"s_subb_u32 {D_QP[1]}, {D_QP[1]}, 0")
        e.salu(f"s_lshl_b32 {D_T}, {'%[qrb]' if self.dropout else '%[orb]'}, 5")
        e.salu(f"s_sub_u32 {D_OP[0]}, {D_OP[0]}, {D_T}")
        e.salu(f"s_subb_u32 {D_OP[1]}, {D_OP[1]}, 0")
        for p0, p1 in (D_LP, D_DP):
            e.salu(f"s_sub_u32 {p0}, {p0}, 128")
            e.salu(f"s_subb_u32 {p1}, {p1}, 0")
        if self.dropout:
            e.salu(f"s_sub_u32 {D_MC}, {D_MC}, %[mstep]")
        e.raw(f"s_branch .Lhp%=_{tag}_adv")
        e.label(f".Lhp%=_{tag}_wrap")
        e.salu(f"s_mov_b32 {D_NMT}, 0")
        e.salu(f"s_mov_b32 {D_NM}, %[mlast]")
        e.salu(f"s_add_u32 {D_QP[0]}, {D_QP[0]}, %[qwrap]")
        e.salu(f"s_addc_u32 {D_QP[1]}, {D_QP[1]}, 0")
        e.salu(f"s_add_u32 {D_OP[0]}, {D_OP[0]}, %[owrap]")
        e.salu(f"s_addc_u32 {D_OP[1]}, {D_OP[1]}, 0")
        for p0, p1 in (D_LP, D_DP):
            e.salu(f"s_add_u32 {p0}, {p0}, %[lwrap]")
            e.salu(f"s_addc_u32 {p1}, {p1}, 0")
        if self.dropout:
            e.salu(f"s_add_u32 {D_MC}, {D_MC}, %[mwrap]")
        e.label(f".Lhp%=_{tag}_adv")

    def dma_items(self, nb, tag):
        """One step's request into buffer nb as (cost, emit) items: the descriptors, wave 0's
        LSE2 / delta rows, the Q, dO pieces (m0 set one item ahead), then the cursors.  Every
        wave's last DK_VMEM vector-memory ops are its pieces."""
        pieces = [("q", 0), ("q", 1), ("o", 0), ("o", 1)]

        def m0_of(w_, it):
            return nb * 16384 + (8192 if w_ == "o" else 0) + it * 4096

        # (issue costs of scalar instructions are taken as 2 cycles each)
        out = [(12, lambda: self.descriptors(0)), (4, lambda: self.descriptors(1))]

        def rows(tag=tag):
            e = self.e
            e.raw("s_cmp_eq_u32 %[w0], 0")
            e.raw(f"s_cbranch_scc0 .Lhp%=_{tag}_nl")
            # one row per lane (lanes 0-31): the range ends exactly at the last row below Lq
            e.salu(f"s_mov_b64 {D_EX}, exec")
            e.salu("s_mov_b32 exec_lo, -1")
            e.salu("s_mov_b32 exec_hi, 0")
            e.salu(f"s_add_u32 m0, %[lbs], {nb * 256}", m0=True)
            e.dma(f"buffer_load_dword %[lsoff], {D_LD}, 0 offen lds")
            e.salu(f"s_add_u32 m0, %[lbs], {nb * 256 + 128}", m0=True)
            e.dma(f"buffer_load_dword %[lsoff], {D_DD}, 0 offen lds")
            e.salu(f"s_mov_b64 exec, {D_EX}")
            e.label(f".Lhp%=_{tag}_nl")
        out.append((16, rows))
        if self.dropout:
            def words(nb=nb):
                # this wave's 64 keep words of the requested step (rows of the tile, key tiles
                # kt0, kt0 + 1: one word per lane)
                e = self.e
                e.salu(f"s_add_u32 m0, {D_WL}, {nb * 1024}", m0=True)
                e.dma(f"buffer_load_dword %[lsoff], {D_MD}, {D_MC} offen lds")
            out.append((8, words))
        for n, (w_, it) in enumerate(pieces):
            def f(n=n, w_=w_, it=it):
                if n == 0:
                    self.e.salu(f"s_add_u32 m0, %[mlds], {m0_of(w_, it)}", m0=True)
                off = f"%[{'q' if w_ == 'q' or self.dropout else 'o'}off{it}]"
                self.e.dma(f"buffer_load_dwordx4 {off}, {D_QD if w_ == 'q' else D_OD}, 0 offen lds")
                if n + 1 < len(pieces):
                    self.e.salu(f"s_add_u32 m0, %[mlds], {m0_of(*pieces[n + 1])}", m0=True)
            out.append((16, f))
        out.append((20, lambda: self.advance_cursors(tag)))
        return out

    def keep_items(self, par, g):
        """Dropout: this step's keep words (buffer par: lane (r32, hh) holds row r32 of key tile
        hh) -> DKM[kb] = the lane's column of key block kb (bit r = row r; the hh = 1 lanes shifted
        by 4 so bit (i & 3) + 8 (i >> 2) is register i's row), as dkdv_kernel's transpose32_lanes:
        five ds_swizzle xor stages within each 32-lane half (the lane-dependent halves of a stage
        under exec masks), then one v_permlane32_swap hands each half the other key block."""
        e = self.e
        m0_, m1_ = DKM
        g.add("tp", 4, -1, 0, lambda: e.ds_read(f"ds_read_b32 {m0_}, %[lsoff] offset:{1024 * par}", m0_),
              lds=1)
        masks = {16: 0x0000FFFF, 8: 0x00FF00FF, 4: 0x0F0F0F0F, 2: 0x33333333, 1: 0x55555555}
        for n, J in enumerate((16, 8, 4, 2, 1)):
            def sw(J=J):
                e._need_lgkm({m0_})
                e.ds_read(f"ds_swizzle_b32 {m1_}, {m0_} offset:{0x1F | (J << 10)}", m1_)

            def stage(J=J):
                e._need_lgkm({m1_})
                e.salu(f"s_mov_b32 s98, {hex(masks[J])}")
                # lanes with lane bit J clear: x = (x & m) | (y << J & ~m)
                e.salu("s_mov_b32 exec_lo, s98")
                e.salu("s_mov_b32 exec_hi, s98")
                e.valu(f"v_lshlrev_b32 {m1_}, {J}, {m1_}", m1_, [m1_])
                e.valu(f"v_bfi_b32 {m0_}, s98, {m0_}, {m1_}", m0_, [m0_, m1_])
                # lanes with it set: x = (y >> J & m) | (x & ~m)
                e.salu("s_not_b32 exec_lo, s98")
                e.salu("s_not_b32 exec_hi, s98")
                e.valu(f"v_lshrrev_b32 {m1_}, {J}, {m1_}", m1_, [m1_])
                e.valu(f"v_bfi_b32 {m0_}, s98, {m1_}, {m0_}", m0_, [m0_, m1_])
                e.salu("s_mov_b64 exec, -1")
            g.add("tp", 4, 2 * n, 2 * n + 2, sw, lds=1)
            g.add("tp", 20, 2 * n + 1, 2 * n + 3, stage)

        def fin():
            e.valu(f"v_mov_b32 {m1_}, {m0_}", m1_, [m0_])
            e.valu(f"v_permlane32_swap_b32 {m0_}, {m1_}", [m0_, m1_], [m0_, m1_], kind="perm")
            e.salu("s_mov_b32 exec_lo, 0")
            e.valu(f"v_lshrrev_b32 {m0_}, 4, {m0_}", m0_, [m0_])
            e.valu(f"v_lshrrev_b32 {m1_}, 4, {m1_}", m1_, [m1_])
            e.salu("s_mov_b64 exec, -1")
        g.add("tp", 20, 10, 12, fin)

    def pack_keep(self, kb, sp, j):
        """Dropout: zero the halves of the P pack PP[kb][sp][j] whose element the forward dropped
        (dV is scaled by 1 / (1 - p) once, in the epilogue)."""
        e = self.e
        pp, t = DPP(kb, sp, j), DTM[kb]
        for h, a in enumerate((8 * sp + 2 * j, 8 * sp + 2 * j + 1)):
            o = (a & 3) + 8 * (a >> 2)
            e.valu(f"v_bfe_i32 {t}, {DKM[kb]}, {o}, 1", t, [DKM[kb]])
            # (SDWA writes the low 16 bits of the result to the selected word: select the same word
            # of both sources; bench_micro/sdwa_test.hip pins this on the hardware)
            e.valu(f"v_and_b32_sdwa {pp}, {t}, {pp} dst_sel:WORD_{h} dst_unused:UNUSED_PRESERVE src0_sel:WORD_{h} "
                   f"src1_sel:WORD_{h}", pp, [t, pp])

    def mask_elem(self, st, kb, i):
        """Causal: P = row >= key - diag ? P : 0 for register i of key block kb, as
        CM + o - kd[kb] >= lr (o = the row offset of the register, kd[kb] = the block's first key
        - diag, lr = r32 - 4 hh).  No other mask: query rows past Lq read zero Q, dO, LSE2 and
        delta (the descriptors' ranges), so P = 1 there multiplies zeros; keys past Lk only reach
        their own dK / dV rows, which are not stored."""
        if not self.causal:
            return
        e = self.e
        o = (i & 3) + 8 * (i >> 2)
        r = DS(st, kb, i)
        # s96 + kb = CM - kd[kb] (mask_bases, at the step start)
        e.salu(f"s_add_u32 s98, s{96 + kb}, {o}")
        e.valu("v_cmp_ge_i32_e32 vcc, s98, %[lr]", None, [])
        e.valu(f"v_cndmask_b32_e32 {r}, 0, {r}, vcc", r, [r])

    def mask_bases(self):
        """s96 + kb = CM - kd[kb] of a masked step (kd[1] = kd[0] + 32)."""
        e = self.e
        e.salu(f"s_sub_u32 s96, {D_CM}, %[kd0]")
        e.salu("s_sub_u32 s97, s96, 32")

    def cvt(self, d, a, b):
        self.e.valu(f"{self.cvtop} {d}, {a}, {b}", d, [a, b])

    # -- MFMAs -----------------------------------------------------------------------------------
    def mf_dk_tail(self, g):
        """Straddled MFMA g (0-7): dK^T[kb][dt] += Q^T(rows 16-31, dt) dS[kb] rows 16-31 of the
        previous step (Q^T fragment in row-ring slot dt)."""
        dt, kb = g >> 1, g & 1
        self.e.mfma(self.mop, DDK(kb, dt), DRR(dt), DDSP(kb, 1), DDK(kb, dt))

    def mf_s(self, st, g):
        """S(next)[kb] (set st) += Q(ks) K[kb](ks), g = 2 ks + kb."""
        ks, kb = g >> 1, g & 1
        self.e.mfma(self.mop, DS(st, kb), DRR(ks), f"%[k{kb * 8 + ks}]", "0" if ks == 0 else DS(st, kb))

    # -- one step --------------------------------------------------------------------------------
    def step(self, ph, cls, tag):
        """Step i with i mod (the layout's phase count) = ph, class A (live, unmasked), B (live, masked) or D (no key
        of the wave visible: only the straddled MFMAs, S(i+1) and the request)."""
        e = self.e
        L = self.L
        par = ph % L.nbuf      # buffer of step i
        st = ph & 1            # S / P set of step i; S(i+1) goes to 1 - st
        nxt = (ph + 1) % L.nbuf
        # half barriers: the even step of a pair requests steps i + 3 and i + 4 (the buffers of
        # steps i - 2 and i - 1, both read before the barrier after step i - 1), the odd one none,
        # so every request has a whole step to land before the barrier (FA2_HPGEN_ABL=dk_hb1: one
        # request per step, the odd step's issued early)
        pair = L.halfbar and "dk_hb1" not in ABL
        early = L.halfbar and not pair and ph & 1
        if pair:
            reqs = [] if ph & 1 else [((par + DK_AHEAD) % L.nbuf, tag), ((par + DK_AHEAD + 1) % L.nbuf, tag + "x")]
        else:
            reqs = [((par + DK_AHEAD) % L.nbuf, tag)]
        live = cls in ("A", "B")
        masked = cls == "B"
        if masked and self.causal:
            self.mask_bases()
        # the MFMAs of the step (indices of `mfma` below): a live step all 64; a dead step (no key of
        # the wave visible) only what a neighbour needs (round 6; round 5 ran the straddled eight and
        # S(i+1) in every dead step: 3.9 % more MFMAs than the algorithm per launch) --
        #   D  (the head's first dead step, also its last): the straddled MFMAs that finish the last
        #      live step's dK, and S(i+1) for the next head's first step;
        #   Ds (first dead step, more follow): the straddled MFMAs only;
        #   E  (neither first nor last): none;
        #   F  (the head's last dead step after others): S(i+1) only
        mf = list(range(64)) if live else {"D": list(range(24)), "Ds": list(range(8)), "E": [],
                                           "F": list(range(8, 24))}[cls]
        if "dk_r5" in ABL and not live:  # A/B reference: round 5's dead steps (24 MFMAs each)
            mf = list(range(24))
        pos = {m: n for n, m in enumerate(mf)}
        last = max(len(mf) - 1, -1)
        g = GapScheduler(len(mf), lds_cap=None if "dk_nocap" in ABL else 3)
        # Q(i+1) row fragments ks -> ring slot ks % 4 (after the slot's previous occupant's last
        # MFMA: the straddled MFMAs 2 dt + kb, then S MFMAs 8 + 2 ks + kb); none without S(i+1)
        if 8 in pos:
            for ks in range(8):
                if 0 in pos:
                    rel, dl = 2 * ks + 1, 2 * ks + 5
                else:
                    # F: no straddled MFMA reads the slots (the step before was Ds or E), so
                    # fragments 0-3 go at once; fragment ks >= 4 reuses slot ks % 4 only after
                    # both S MFMAs of fragment ks - 4 have read it
                    rel = -1 if ks < 4 else pos[8 + 2 * (ks - 4) + 1] + 1
                    dl = max(rel, pos[8 + 2 * ks] - 3)
                g.add("row", 4, rel, dl, lambda ks=ks: self.row_read(nxt, False, ks), lds=2)
        items = [it for nb, t in reqs for it in self.dma_items(nb, t)]
        for n, (c, f) in enumerate(items):
            if pair:
                dl = min(20 + 3 * n, 62) if live else min(6 + n, last)
            else:
                dl = (20 if early and live else 42 if live else 14) + 3 * n
                dl = dl if live else min(dl, last)
            g.add("dma", c, 0 if early or not live else 2, dl, f)
        if live:
            # dO(i) row fragments ks (slot ks % 4, after the S MFMAs 2 ks + 17), dP at 24 + 2 ks
            for ks in range(8):
                rel = 2 * ks + 17
                g.add("row", 4, rel, rel + 4, lambda ks=ks: self.row_read(par, True, ks), lds=2)
            # Q^T(i) fragments of rows 16-31 (f = 4 + dt) into row-ring slots dt, after the dP
            # MFMAs that read the slot's dO fragment (2 dt + 33): the next step's first MFMAs
            for dt in range(4):
                for h in range(2):
                    g.add("row", 4, 2 * dt + 33, 58,
                          lambda dt=dt, h=h: self.tr_read(par, False, 4 + dt, h, DRR(dt, h)), lds=1)
            # V fragments n (slot n % 4): dP MFMA 24 + n
            for n in range(16):
                rel = 8 if n < self.vslots else 24 + n - self.vslots
                g.add("vf", 4, rel, max(rel, 21 + n), lambda n=n: self.v_frag(n), lds=2)
            # dO^T fragments f (slot f % 4): dV MFMAs 40 + 2 f + kb; then Q^T rows 0-15 (slot f)
            for f in range(8):
                rel = 0 if f < 4 else 2 * f + 33
                for h in range(2):
                    g.add("tr", 4, rel, 2 * f + 37, lambda f=f, h=h: self.tr_read(par, True, f, h, DTR(f, h)), lds=1)
            for f in range(4):
                for h in range(2):
                    g.add("tr", 4, 2 * f + 49, 2 * f + 53, lambda f=f, h=h: self.tr_read(par, False, f, h, DTR(f, h)),
                          lds=1)
            # -delta rows into dP[1] only (register groups g4; g4 = 2 holds the packed dS of rows
            # 16-31 that the straddled MFMAs 2 dt + 1 read: after them); the first dP MFMA of block
            # 0 takes dP[1] as its C (before block 1's chain overwrites it), so both chains start
            # from the one copy of the rows
            if not self.dropout:
                for g4 in range(4):
                    g.add("init1", 4, 8 if g4 == 2 else 0, 20, lambda g4=g4: self.init_read(par, 1, 1, g4), lds=2)
            else:
                # -delta rows (group g4) for dS = P (dP kp - delta), into V ring slot g4 once the
                # dP MFMA 36 + g4 has read it
                for g4 in range(4):
                    d = DDEL(g4)
                    rel, dl = 36 + g4, 41 + g4
                    g.add("dl", 4, rel, dl, lambda g4=g4, d=d: self.e.ds_read(
                        f"ds_read_b128 {d}, %[lb] offset:{par * 256 + 128 + 32 * g4}", d), lds=2)
                self.keep_items(par, g)
            # LSE2 of this step's half sp = 1 once every sp = 0 exponent argument is done; half
            # sp = 0 of the NEXT step once every sp = 1 one is (its rows landed a step ago), so no
            # exponential waits for an LDS read at a step start (round 5: that wait cost ~8 %)
            for g4 in (2, 3):
                g.add("lse", 4, 14, 18, lambda g4=g4: self.init_read(par, 0, 0, g4), lds=2)
            for g4 in (0, 1):
                g.add("lse", 4, 40, 58, lambda g4=g4: self.init_read(nxt, 0, 0, g4), lds=2)
            # exponentials of P(i) (set st): P = exp2(s scale log2 e - LSE2), the scale in fp32;
            # mask; packs PP[kb][sp] (dV MFMAs 40 + 8 sp + 2 dt + kb)
            for sp in range(2):
                r0, r1 = (0, 18) if sp == 0 else (21, 44)
                for kb in range(2):
                    els = list(range(8 * sp, 8 * sp + 8))
                    for k, i in enumerate(els):
                        r = DS(st, kb, i)
                        dl = r0 + ((r1 - r0 - 6) * (k + 1)) // 8
                        g.add(f"exp{kb}", 4, r0, dl,
                              lambda r=r, i=i: e.valu(f"v_fma_f32 {r}, {r}, %[sc], -{DLSE(i)}", r, [r, DLSE(i)]))
                        g.add(f"exp{kb}", 8, r0, dl + 1, lambda r=r: e.valu(f"v_exp_f32 {r}, {r}", r, [r], kind="trans"))
                        if masked and self.causal:
                            g.add(f"exp{kb}", 12, r0, dl + 2, lambda kb=kb, i=i: self.mask_elem(st, kb, i))
                    for j in range(4):
                        g.add(f"exp{kb}", 4, r0, (38 if sp == 0 else (42 if self.dropout else 46)),
                              lambda kb=kb, sp=sp, j=j: self.cvt(DPP(kb, sp, j), DS(st, kb, 8 * sp + 2 * j),
                                                               DS(st, kb, 8 * sp + 2 * j + 1)))
                        if self.dropout:  # (the keep columns are ready after the transposition;
                            # DTM[kb] is the dS side's from MFMA 43 on)
                            g.add(f"exp{kb}", 16, max(r0, 13), (38 if sp == 0 else 42),
                                  lambda kb=kb, sp=sp, j=j: self.pack_keep(kb, sp, j))
            # dS(i) = P dP' after the dP chains (last MFMA 39; 4 MFMAs for the result), packs in place; DSP[kb][0] for the
            # MFMAs 56 + 2 dt + kb, DSP[kb][1] for the next step's first MFMAs
            for kb in range(2):
                if self.dropout:
                    # dS = P (dP kp - delta), kp = keep ? 1 / (1 - p) : 0 (bit for bit dkdv_kernel's
                    # pr * (dp * kp + d4)); by row group g4, packs j of the group right after it
                    for g4 in range(4):
                        sp, dl = g4 >> 1, (50, 53, 58, 61)[g4]
                        for i in range(4 * g4, 4 * g4 + 4):
                            a_, b_, t_, d_ = DS(st, kb, i), DDP(kb, i), DTM[kb], DDEL(g4, i & 3)
                            o = (i & 3) + 8 * (i >> 2)

                            def dsd(a_=a_, b_=b_, t_=t_, d_=d_, o=o, kb=kb):
                                e.valu(f"v_bfe_i32 {t_}, {DKM[kb]}, {o}, 1", t_, [DKM[kb]])
                                e.valu(f"v_and_b32 {t_}, %[dscb], {t_}", t_, [t_])
                                e.valu(f"v_fma_f32 {b_}, {b_}, {t_}, {d_}", b_, [b_, t_, d_])
                            g.add(f"ds{kb}", 12, 43, dl, dsd)
                            g.add(f"ds{kb}", 4, 43, dl,
                                  lambda a_=a_, b_=b_: e.valu(f"v_mul_f32 {b_}, {a_}, {b_}", b_, [a_, b_]))
                        for j in (2 * (g4 & 1), 2 * (g4 & 1) + 1):
                            g.add(f"ds{kb}", 4, 43, dl + 1,
                                  lambda kb=kb, sp=sp, j=j: self.cvt(DDSP(kb, sp, j), DDP(kb, 8 * sp + 2 * j),
                                                                   DDP(kb, 8 * sp + 2 * j + 1)))
                    continue
                for sp in range(2):
                    dl = 52 if sp == 0 else 61
                    for i in range(8 * sp, 8 * sp + 8):
                        a_, b_ = DS(st, kb, i), DDP(kb, i)
                        if "dk_pk" in ABL:  # (A/B: dS of element pairs by v_pk_mul_f32)
                            if not i & 1:
                                a2, b2 = rng("v", int(a_[1:]), 2), rng("v", int(b_[1:]), 2)
                                g.add(f"ds{kb}", 8, 43, dl,
                                      lambda a2=a2, b2=b2: e.valu(f"v_pk_mul_f32 {b2}, {a2}, {b2}", b2, [a2, b2]))
                            continue
                        g.add(f"ds{kb}", 4, 43, dl, lambda a_=a_, b_=b_: e.valu(f"v_mul_f32 {b_}, {a_}, {b_}", b_, [a_, b_]))
                    for j in range(4):
                        g.add(f"ds{kb}", 4, 43, dl + 1,
                              lambda kb=kb, sp=sp, j=j: self.cvt(DDSP(kb, sp, j), DDP(kb, 8 * sp + 2 * j), DDP(kb, 8 * sp + 2 * j + 1)))
        else:
            # no dS of this step: the next step's straddled MFMAs add zeros (after this step's
            # straddled MFMAs, which read the packs)
            for kb in range(2):
                for j in range(4):
                    r = DDSP(kb, 1, j)
                    g.add("zero", 4, (7 + kb) if 0 in pos else -1, min(20, last), lambda r=r: e.valu(f"v_mov_b32 {r}, 0", r))
            for g4 in (0, 1):  # the next step's LSE2 of half sp = 0
                g.add("lse", 4, -1, min(20, last), lambda g4=g4: self.init_read(nxt, 0, 0, g4), lds=2)

        if "dk_novalu" in ABL:
            g.items = [it for it in g.items if not it["stream"].startswith(("exp", "ds"))]
        if "dk_nodma" in ABL:
            g.items = [it for it in g.items if it["stream"] != "dma"]
        if "dk_nolds" in ABL:
            g.items = [it for it in g.items if it["stream"] not in ("row", "vf", "tr", "init1", "lse")]
        if "dk_nolgkm" in ABL:
            e.ds = []
            e._need_lgkm = lambda regs: None
        drops = {"dk_noexp": r"^v_exp", "dk_nocvt": r"^v_cvt_pk", "dk_notr": r"^ds_read_b64_tr",
                 "dk_novf": r"%\[vb[01]\]", "dk_norow": r"^ds_read_b128 .*%\[qb[01]\]", "dk_noinit": r"%\[lb\]",
                 "dk_nosalu": r"^s_(mov_b32 s(6[89]|7\d|8[0-3])|and_b32 s|mul_i32|add_u32 s(7[6-9]|8[0-3])|addc|sub_u32 s8[4-9]|subb|cselect|sub_i32)",
                 "dk_nomul": r"^v_mul_f32", "dk_nofma": r"^v_fma_f32",
                 "dk_nolse": r"%\[lb\] offset:(0|32|64|96|256|288|320|352|512|544|576|608|768|800|832|864)$",
                 "dk_nodl": r"%\[lb\] offset:(128|160|192|224|384|416|448|480|640|672|704|736|896|928|960|992)$"}
        pat = "|".join(v for k, v in drops.items() if k in ABL)
        e.drop = re.compile(pat) if pat else None

        def mfma(n):
            m = mf[n]
            if m < 8:
                self.mf_dk_tail(m)
            elif m < 24:
                self.mf_s(1 - st, m - 8)
            elif m < 40:  # dP[kb] += dO(ks) V[kb](ks), both chains seeded from dP[1]'s -delta rows
                ks, kb = (m - 24) >> 1, m & 1
                c = ("0" if self.dropout else DDP(1)) if ks == 0 else DDP(kb)
                e.mfma(self.mop, DDP(kb), DRR(ks), self.dvf(2 * ks + kb), c)
            elif m < 56:  # dV^T[kb][dt] += dO^T(sp, dt) P[kb](sp)
                f, kb = (m - 40) >> 1, m & 1
                e.mfma(self.mop, DDV(kb, f & 3), DTR(f), DPP(kb, f >> 2), DDV(kb, f & 3))
            else:  # dK^T[kb][dt] += Q^T(rows 0-15, dt) dS[kb](rows 0-15)
                f, kb = (m - 56) >> 1, m & 1
                e.mfma(self.mop, DDK(kb, f), DTR(f), DDSP(kb, 0), DDK(kb, f))

        g.run(mfma, pre_budget=24)
        if "dk_nolgkm" in ABL:
            e._need_lgkm = Emitter._need_lgkm.__get__(e)
        e.drop = None
        e.salu(f"s_sub_u32 {D_CM}, {D_CM}, 32")
        e.drain_lds()
        if L.halfbar:
            if ph & 1:
                # every request so far (up to step i + 3) has landed
                e.raw("s_waitcnt vmcnt(0)")
                e.raw("s_barrier")
            else:
                return  # (no reset: the odd step starts from this end state, DkdvGen.build)
        else:
            if "dk_novm" not in ABL:
                # the next step's tiles (requested two steps ago) have landed; this step's stay in
                # flight
                e.raw(f"s_waitcnt vmcnt({DK_VMEM})")
            if "dk_nobar" not in ABL:
                e.raw("s_barrier")
        e.reset()

    def build(self):
        e = self.e
        e.raw("s_nop 7")
        e.raw("s_nop 7")
        e.salu(f"s_mov_b32 {D_M0}, m0")
        for r in range(256):
            e.valu(f"v_accvgpr_write_b32 a{r}, 0", f"a{r}", kind="accw")
        # the first step's straddled MFMAs add zeros
        for kb in range(2):
            for j in range(4):
                e.valu(f"v_mov_b32 {DDSP(kb, 1, j)}, 0", DDSP(kb, 1, j))
        # cursors: step 0's tiles were requested before the statement (and waited for by the
        # compiler's wait for the K fragments); steps 1 and 2 here, then the loop requests step
        # i + 3 during step i
        e.salu(f"s_mov_b32 {D_QP[0]}, %[qlo]")
        e.salu(f"s_mov_b32 {D_QP[1]}, %[qhi]")
        e.salu(f"s_mov_b32 {D_OP[0]}, %[olo]")
        e.salu(f"s_mov_b32 {D_OP[1]}, %[ohi]")
        for (p0, p1), b in ((D_LP, "lse"), (D_DP, "dl")):
            e.salu(f"s_add_u32 {p0}, %[{b}lo], %[lc0]")
            e.salu(f"s_addc_u32 {p1}, %[{b}hi], 0")
        for d in (71, 75, 79, 83):
            e.salu(f"s_mov_b32 s{d}, 0x20000")
        if self.dropout:
            e.salu("s_mov_b32 s84, %[mlo]")
            e.salu("s_mov_b32 s85, %[mhi]")
            e.salu("s_mov_b32 s86, %[mrange]")  # the mask's bytes from the base: reads past it give 0
            e.salu("s_mov_b32 s87, 0x20000")
            # sb + w0 + 256 w (lbs = sb + rows)
            e.salu(f"s_lshl_b32 {D_WL}, %[w0], 8")
            e.salu(f"s_add_u32 {D_WL}, {D_WL}, %[lbs]")
            e.salu(f"s_add_u32 {D_WL}, {D_WL}, {self.L.w0 - self.L.rows}")
        e.salu(f"s_mov_b32 {D_NM}, %[mlast]")
        e.salu(f"s_mov_b32 {D_NMT}, 0")
        e.salu(f"s_mul_i32 {D_LEFT}, %[ng], %[nmt]")  # the block's steps
        if self.dropout:  # step 0's keep words: mstep (nmt - 1)
            e.salu(f"s_sub_u32 {D_MC}, %[nmt], 1")
            e.salu(f"s_mul_i32 {D_MC}, {D_MC}, %[mstep]")
        self.advance_cursors("init")  # -> step 1 (D_LEFT = total - 1)
        # this block's V rows, step-0 tiles and K fragments (requested before the statement, during
        # the previous block's epilogue) have landed; every wave is past that epilogue, whose
        # staging images sit in step buffers 2-3
        e.raw("s_waitcnt vmcnt(0) lgkmcnt(0)")
        e.raw("s_barrier")
        e.reset()
        for nb in (1, 2):
            for _, f in self.dma_items(nb, f"pro{nb}"):
                f()
        e.salu(f"s_mov_b32 {D_G}, 0")
        # no step at all (ng nmt = 0; D_G = 0 here)
        e.raw(f"s_cmp_eq_u32 {D_G}, %[ng]")
        e.raw("s_cbranch_scc1 .Lhp%=_end")
        e.raw("s_cmp_eq_u32 %[nmt], 0")
        e.raw("s_cbranch_scc1 .Lhp%=_end")
        # S(0) into set 0 from buffer 0
        for ks in range(3):
            self.row_read(0, False, ks)
        for m in range(16):
            ks = m >> 1
            if m & 1 and ks + 3 < 8:
                self.row_read(0, False, ks + 3)
            self.mf_s(0, m)
        for g4 in (0, 1):  # step 0's LSE2 of half sp = 0 (each step loads the next one's)
            self.init_read(0, 0, 0, g4)
        e.drain_lds()
        e.drain_mfma()
        # step 1's tiles (half barriers: step 2's too; steps 0 and 1 run before the next barrier)
        e.raw(f"s_waitcnt vmcnt({0 if self.L.halfbar else DK_VMEM})")
        e.raw("s_barrier")
        e.reset()
        e.salu(f"s_mov_b32 {D_IDX}, 0")
        e.salu(f"s_mov_b32 {D_CM}, %[mlast]")
        # one entry per step phase ph: the class of step IDX ([0, c0) B, [c0, c01) A, [c01, c012)
        # B, then D) -> the body (class, ph); each body continues at the entry of phase ph + 1 (the
        # phase is static: no dispatch on it)
        for ph in range(self.L.ph):
            e.raw(".balignl 64, 0xbf800000", 0)
            e.label(f".Lhp%=_step{ph}")
            e.raw(f"s_cmp_lt_u32 {D_IDX}, %[c0]")
            e.raw(f"s_cbranch_scc1 .Lhp%=_B{ph}")
            e.raw(f"s_cmp_lt_u32 {D_IDX}, %[c01]")
            e.raw(f"s_cbranch_scc1 .Lhp%=_A{ph}")
            e.raw(f"s_cmp_lt_u32 {D_IDX}, %[c012]")
            e.raw(f"s_cbranch_scc1 .Lhp%=_B{ph}")
            # dead steps: D / Ds at IDX == c012 (with / without more after it), E between, F last
            e.salu(f"s_add_u32 {D_T}, {D_IDX}, 1")
            e.raw(f"s_cmp_eq_u32 {D_IDX}, %[c012]")
            e.raw(f"s_cbranch_scc0 .Lhp%=_nd{ph}")
            e.raw(f"s_cmp_lt_u32 {D_T}, %[nmt]")
            e.raw(f"s_cbranch_scc1 .Lhp%=_Ds{ph}")
            e.raw(f"s_branch .Lhp%=_D{ph}")
            e.label(f".Lhp%=_nd{ph}")
            e.raw(f"s_cmp_lt_u32 {D_T}, %[nmt]")
            e.raw(f"s_cbranch_scc1 .Lhp%=_E{ph}")
            e.raw(f"s_branch .Lhp%=_F{ph}")
        snaps = []
        for ph in range(self.L.ph):
            ends = []
            for cls in ("A", "B", "D", "Ds", "E", "F"):
                nph = (ph + 1) % self.L.ph
                e.label(f".Lhp%=_{cls}{ph}")
                # half barriers: an odd step follows any of the previous phase's bodies with no
                # barrier between (their merged end states); an even one follows a barrier
                if self.L.halfbar and ph & 1:
                    e.restore(snaps)
                else:
                    e.reset()
                self.step(ph, cls, f"{cls.lower()}{ph}")
                if self.L.halfbar and not ph & 1:
                    if cls not in ("A", "B"):  # (rare: a head's dead steps)
                        e.close_windows()
                    ends.append(e.snapshot())
                # next step: within the head, else the next head's first (IDX 0, CM = mlast)
                e.salu(f"s_add_u32 {D_IDX}, {D_IDX}, 1")
                e.raw(f"s_cmp_lt_u32 {D_IDX}, %[nmt]")
                e.raw(f"s_cbranch_scc1 .Lhp%=_step{nph}")
                e.salu(f"s_add_u32 {D_G}, {D_G}, 1")
                e.salu(f"s_mov_b32 {D_IDX}, 0")
                e.salu(f"s_mov_b32 {D_CM}, %[mlast]")
                e.raw(f"s_cmp_lt_u32 {D_G}, %[ng]")
                e.raw(f"s_cbranch_scc1 .Lhp%=_step{nph}")
                e.raw("s_branch .Lhp%=_last")
            snaps = ends
        e.label(".Lhp%=_last")
        # (after any body: every window closed)
        e.ds = []
        e._pad(max(Emitter.MFMA_RESULT, Emitter.MFMA_C_WAR))
        e.reset()
        # the last step's straddled MFMAs
        for m in range(8):
            self.mf_dk_tail(m)
        e.label(".Lhp%=_end")
        # every wave's (range-0) requests of the last steps have landed before any wave stages
        # its epilogue in the step buffers
        e.raw("s_waitcnt vmcnt(0) lgkmcnt(0)")
        e.raw("s_barrier")
        e.salu(f"s_mov_b32 m0, {D_M0}")
        e.raw("s_nop 15")
        e.raw("s_nop 15")
        return e.out


def gen_dkdv_function(bf16, causal, dropout=False):
    g = DkdvGen(bf16, causal, dropout)
    lines = g.build()
    name = f"dkdv_hp_main_{'bf16' if bf16 else 'f16'}_{'causal' if causal else 'full'}{'_drop' if dropout else ''}"
    clob = [f'"v{i}"' for i in range(g.nvgpr)] + [f'"a{i}"' for i in range(256)] + \
           [f'"s{i}"' for i in _sgprs_used(lines)] + ['"vcc"', '"scc"', '"memory"']
    kops = ", ".join(f'[k{i}] "v"(kf[{i}])' for i in range(16))
    sops = ["ng", "nmt", "c0", "c01", "c012", "mlast", "lq", "qrb"] + ([] if dropout else ["orb"]) + ["qwrap",
            "owrap", "lwrap", "lc0", "qlo", "qhi", "olo", "ohi", "lselo", "lsehi", "dllo", "dlhi", "mlds", "lbs", "w0",
            "sc"] + (["kd0"] if causal else []) + (["mlo", "mhi", "mrange", "mstep", "mwrap"] if dropout else [])
    vops = ["qb0", "qb1", "vb0", "vb1", "ta", "tb"] + (["qb0h", "qb1h", "tah", "tbh"] if g.L.nbuf > 4 else []) + ["lb", "qoff0", "qoff1"] + ([] if dropout else ["ooff0", "ooff1"]) + \
        ["lsoff"] + (["lr"] if causal else []) + (["dscb"] if dropout else [])
    src = f"""// hand-placed dK/dV statement ({'bf16' if bf16 else 'fp16'}, {'causal' if causal else 'non-causal'}): {len(lines)} lines, {g.e.n_mfma} MFMAs
FA2_DEV void {name}(const u32x4 (&kf)[16], const DkdvHpArgs& a) {{
  asm volatile(
{_asm_body(lines)}
      :
      : {kops},
        {", ".join(f'[{n}] "v"(a.{n})' for n in vops)},
        {", ".join(f'[{n}] "s"(a.{n})' for n in sops)}
      : {", ".join(clob)});
}}
"""
    return src


def gen_read_dkdv():
    parts = ["// dV^T a[0:127], dK^T a[128:255] of key block KB -> registers (after the statement's final",
             "// drain); one key block at a time keeps the epilogue within the register file; tok: a",
             "// value of the next block's requests (kept ahead of these reads by the data dependence)",
             "template <int KB>",
             "FA2_DEV void dkdv_hp_read(f32x16 (&dv)[4], f32x16 (&dk)[4], uint32_t tok);"]
    for kb in range(2):
        parts.append("template <>")
        parts.append(f"FA2_DEV void dkdv_hp_read<{kb}>(f32x16 (&dv)[4], f32x16 (&dk)[4], uint32_t tok) {{")
        for which, base0 in (("dv", 0), ("dk", 128)):
            for dt in range(4):
                base = base0 + (kb * 4 + dt) * 16
                outs = ", ".join(f'"=v"({which}[{dt}][{i}])' for i in range(16))
                body = "".join(f"v_accvgpr_read_b32 %{i}, a{base + i}\\n" for i in range(16))
                clob = ", ".join(f'"a{r}"' for r in range(256))
                parts.append(f'  asm volatile("{body}" : {outs} : "s"(tok) : {clob});')
        parts.append("}")
    return "\n".join(parts) + "\n"



# ----------------------------------------------------------------------------------------------
# dQ: dq_hp_kernel (csrc/dq_hp_kernel.h)
#
# Register map of the statement:
#   v[0:63]     S^T[rb][h] (scores of key half h; then P), v[64:127] dP^T[rb][h] (then dS, then
#               in place the packed dS^T DSP[rb][kk]: the B operands of dQ^T += K^T dS^T)
#   v[128:143]  K row-fragment ring, v[144:159] V row-fragment ring, v[160:175] K^T ring
#   v[176:177]  mask limits of a masked tile
#   a[0:127]    dQ^T[rb][dt]; a[128:255] the Q and dO fragments ("a" operands)
def QS(rb, h, i=None):
    base = (rb * 2 + h) * 16
    return rng("v", base, 16) if i is None else f"v{base + i}"


def QDP(rb, h, i=None):
    base = 64 + (rb * 2 + h) * 16
    return rng("v", base, 16) if i is None else f"v{base + i}"


def QDSP(rb, kk, j=None):
    """Packed dS^T of 16-key step kk, in place over dP^T[rb][kk >> 1]: pack j of the 8-element
    group 8 (kk & 1) .. + 7 reads elements 2j, 2j + 1 and writes element j (consumed by pack j // 2,
    issued before it in the same stream), so the four packs land in consecutive registers."""
    base = 64 + (rb * 2 + (kk >> 1)) * 16 + 8 * (kk & 1)
    return rng("v", base, 4) if j is None else f"v{base + j}"


def QKR(n):
    return rng("v", 128 + 4 * (n % 4), 4)


def QVR(n):
    return rng("v", 144 + 4 * (n % 4), 4)


def QTR(n, half=None):
    base = 160 + 4 * (n % 4)
    return rng("v", base, 4) if half is None else rng("v", base + 2 * half, 2)


QREL = ["v176", "v177"]
# round 6 (no dropout): -delta of the lane's row in all 16 registers of a block per row block: the
# C operand of the first dP MFMA of both key halves, so the chain yields dP - delta and dS is one
# multiply (as dkdv_hp; dq_kernel seeds its chain the same way, the two stay bitwise equal)


def QNDEL(rb):
    return rng("v", 178 + 16 * rb, 16)


DQ_NVGPR = 178
# dropout (the forward's saved keep words, one 32-key word per row): the words of the current and
# the next tile, per (rb, key half h); per-stream temporaries; the lane's word offsets (cursor)
def QMW(st, rb, h):
    return f"v{DQ_NVGPR + 4 * st + 2 * rb + h}"


def QMT(h, rb):
    """dS temporaries: the K ring's slot 0, free once the S chains are issued (the dS phase
    starts 18 MFMAs later)."""
    return f"v{128 + 2 * h + rb}"


QMO = f"v{DQ_NVGPR + 8}"  # lane byte offset of row block 0's tile-0 words (row block 1: + %[mrs])
DQ_NVGPR_DROP = DQ_NVGPR + 9
Q_MD = "%[mdesc]"  # keep-word descriptor (a 4-SGPR operand)
Q_MOFF = ["s96", "s97"]  # byte offsets of the requested tile's words, row block 0 / 1


def QDQ(rb, dt):
    return rng("a", (rb * 4 + dt) * 16, 16)


# scalar state of the dQ statement (shares the forward's cursor registers)
Q_SN0 = "s66"  # first key of the current tile
Q_PAR = "s67"  # buffer parity of the current tile: (i + boff) & 1
Q_FIN = "s83"  # index of the unit's final tile
Q_NA = "s84"   # class A tiles the A chain runs: min(na, final)


class DqGen:
    """dQ (recompute form, deterministic): 4 waves x 64 query rows (two 32-row blocks rb per
    wave, one wave per SIMD); per 64-key tile 96 MFMAs: S^T = K Q'^T (32), dP^T = V dO^T (32),
    dQ^T += K^T dS^T (32); every K, V and K^T fragment read from LDS feeds both row blocks.
    Same math as the reference's dQ loop (/root/reference/src/backward/compute_dq.py:38-78)
    and dq_kernel: P = exp2(s scale log2 e - LSE2), dS = P (dP - delta), dQ = scale dS K."""

    def __init__(self, bf16, causal, dropout=False):
        self.bf16, self.causal, self.dropout = bf16, causal, dropout
        self.seed = not dropout and "dq_r5" not in ABL  # dP chains seeded with -delta (QNDEL)
        self.mop = "v_mfma_f32_32x32x16_bf16" if bf16 else "v_mfma_f32_32x32x16_f16"
        self.cvtop = "v_cvt_pk_bf16_f32" if bf16 else "v_cvt_pk_f16_f32"
        self.e = Emitter()

    def mask_items(self, par):
        """Dropout: the keep words of the next tile (rows of rb, keys 32 h ..) into set 1 - par;
        four dword loads, then the cursor moves one tile (64 keys = 2 words = 256 bytes per row
        block tile of 32 rows)."""
        e = self.e
        out = []
        for rb in range(2):
            for h in range(2):
                def f(rb=rb, h=h):
                    e.raw(f"buffer_load_dword {QMW(1 - par, rb, h)}, {QMO}, {Q_MD}, {Q_MOFF[rb]} offen offset:{128 * h}")
                    if rb == 1 and h == 1:
                        e.salu(f"s_add_u32 {Q_MOFF[0]}, {Q_MOFF[0]}, 256")
                        e.salu(f"s_add_u32 {Q_MOFF[1]}, {Q_MOFF[1]}, 256")
                out.append((16, f))
        return out

    def k_read(self, par, n):
        h, ks = n // 8, n % 8
        imm = par * 16384 + (ks >> 1) * 4096 + 32 * h * 64
        d = QKR(n)
        self.e.ds_read(f"ds_read_b128 {d}, {'%[kb1]' if ks & 1 else '%[kb0]'} offset:{imm}", d)

    def v_read(self, par, n):
        h, ks = n // 8, n % 8
        imm = 32768 + par * 16384 + (ks >> 1) * 4096 + 32 * h * 64
        d = QVR(n)
        self.e.ds_read(f"ds_read_b128 {d}, {'%[kb1]' if ks & 1 else '%[kb0]'} offset:{imm}", d)

    def t_read(self, par, n, half):
        kk, dt = n // 4, n % 4
        imm = par * 16384 + dt * 4096 + 16 * kk * 64
        d = QTR(n, half)
        self.e.ds_read(f"ds_read_b64_tr_b16 {d}, {'%[tb]' if half else '%[ta]'} offset:{imm}", d)

    def descriptors(self):
        FwdGen.descriptors(self)

    def dma_items(self, par):
        """K(i+1), V(i+1) into buffer 1 - par (m0 one item ahead)."""
        nb = 1 - par
        pieces = [("k", it) for it in range(4)] + [("v", it) for it in range(4)]

        def m0_of(w_, it):
            return nb * 16384 + it * 4096 + (32768 if w_ == "v" else 0)

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

    def mask_elem(self, rb, h, i):
        """P = key offset o < REL[rb] ? P : 0 (o = 32 h + (i & 3) + 8 (i >> 2))."""
        e = self.e
        o = 32 * h + (i & 3) + 8 * (i >> 2)
        r = QS(rb, h, i)
        sm = SMASK[i & 1]
        e.valu(f"v_cmp_gt_i32_e64 {sm}, {QREL[rb]}, {o}", None, [QREL[rb]])
        e.valu(f"v_cndmask_b32_e64 {r}, 0, {r}, {sm}", r, [r])

    def cvt(self, d, a, b):
        self.e.valu(f"{self.cvtop} {d}, {a}, {b}", d, [a, b])

    def period(self, par, cls):
        e = self.e
        self.descriptors()
        dma = self.dma_items(par) + (self.mask_items(par) if self.dropout else [])
        if cls == "D":
            for _, f in dma:
                f()
        else:
            masked = cls == "B"
            if masked:
                for rb in range(2):
                    e.valu(f"v_subrev_u32 {QREL[rb]}, {Q_SN0}, %[rel{rb}]", QREL[rb], [])
            g = GapScheduler(96)
            for n in range(16):  # K row fragments, then V row fragments: 3 ahead (ring of 4)
                mf = 2 * n
                rel = -1 if n < 3 else mf - 6
                g.add("k", 4, rel, max(rel, mf - 4), lambda n=n: self.k_read(par, n))
            for n in range(16):
                mf = 32 + 2 * n
                rel = max(-1, mf - 6)
                g.add("v", 4, rel, mf - 4, lambda n=n: self.v_read(par, n))
            for n in range(16):  # K^T fragments for dQ: 3 ahead
                mf = 64 + 2 * n
                for hf in range(2):
                    g.add("t", 4, mf - 6, mf - 3, lambda n=n, hf=hf: self.t_read(par, n, hf))
            for h in range(2):
                rel0 = 18 + 16 * h
                for rb in range(2):
                    for i in range(16):
                        r = QS(rb, h, i)
                        st = f"p{h}{rb}"
                        g.add(st, 4, rel0, 38 + 16 * h,
                              lambda r=r, rb=rb: e.valu(f"v_fma_f32 {r}, {r}, %[sc], -%[lse{rb}]", r, [r]))
                        g.add(st, 8, rel0, 40 + 16 * h, lambda r=r: e.valu(f"v_exp_f32 {r}, {r}", r, [r], kind="trans"))
                        if masked:
                            g.add(st, 8, rel0, 41 + 16 * h, lambda rb=rb, h=h, i=i: self.mask_elem(rb, h, i))
                rel1 = 50 + 16 * h
                for rb in range(2):
                    if self.dropout:  # this lane's keys start 4 hh into the word
                        w_ = QMW(par, rb, h)
                        g.add(f"d{h}{rb}", 4, -1, rel1,
                              lambda w_=w_: e.valu(f"v_lshrrev_b32 {w_}, %[msh], {w_}", w_, [w_]))
                    for i in range(16):
                        a_, b_ = QS(rb, h, i), QDP(rb, h, i)
                        st = f"d{h}{rb}"
                        if self.dropout:
                            # dS = P (dP M / (1 - p) - delta), M the forward's keep bit
                            t_, w_, k_ = QMT(h, rb), QMW(par, rb, h), (i & 3) + 8 * (i >> 2)
                            g.add(st, 4, rel1, 56 + 16 * h,
                                  lambda t_=t_, w_=w_, k_=k_: e.valu(f"v_bfe_i32 {t_}, {w_}, {k_}, 1", t_, [w_]))
                            g.add(st, 4, rel1, 57 + 16 * h,
                                  lambda t_=t_, b_=b_: e.valu(f"v_and_b32 {b_}, {t_}, {b_}", b_, [t_, b_]))
                            g.add(st, 4, rel1, 58 + 16 * h,
                                  lambda b_=b_, rb=rb: e.valu(f"v_fma_f32 {b_}, {b_}, %[dsc], -%[del{rb}]", b_, [b_]))
                        elif not self.seed:  # (A/B reference, FA2_HPGEN_ABL=dq_r5)
                            g.add(st, 4, rel1, 58 + 16 * h,
                                  lambda b_=b_, rb=rb: e.valu(f"v_sub_f32 {b_}, {b_}, %[del{rb}]", b_, [b_]))
                        if "dq_pk" in ABL and self.seed:  # (A/B: dS of element pairs by v_pk_mul_f32)
                            if not i & 1:
                                a2, b2 = rng("v", int(a_[1:]), 2), rng("v", int(b_[1:]), 2)
                                g.add(st, 8, rel1, 60 + 16 * h,
                                      lambda a2=a2, b2=b2: e.valu(f"v_pk_mul_f32 {b2}, {a2}, {b2}", b2, [a2, b2]))
                        else:
                            g.add(st, 4, rel1, 60 + 16 * h, lambda a_=a_, b_=b_: e.valu(f"v_mul_f32 {b_}, {a_}, {b_}", b_, [a_, b_]))
                        if i & 1:
                            kk, j = 2 * h + (i >> 3), (i & 7) >> 1
                            g.add(st, 4, rel1, 62 + 16 * h,
                                  lambda rb=rb, kk=kk, j=j, h=h, i=i: self.cvt(QDSP(rb, kk, j), QDP(rb, h, i - 1), QDP(rb, h, i)))
            for n, (c, f) in enumerate(dma):
                g.add("dma", c, 0, 40 + 4 * n, f)

            def mfma(gi):
                if gi < 32:
                    h, ks, rb = gi >> 4, (gi >> 1) & 7, gi & 1
                    d = QS(rb, h)
                    e.mfma(self.mop, d, QKR(8 * h + ks), f"%[q{rb * 8 + ks}]", "0" if ks == 0 else d)
                elif gi < 64:
                    x = gi - 32
                    h, ks, rb = x >> 4, (x >> 1) & 7, x & 1
                    d = QDP(rb, h)
                    c0 = QNDEL(rb) if self.seed else "0"
                    e.mfma(self.mop, d, QVR(8 * h + ks), f"%[o{rb * 8 + ks}]", c0 if ks == 0 else d)
                else:
                    f_, rb = (gi - 64) >> 1, gi & 1
                    kk, dt = f_ >> 2, f_ & 3
                    e.mfma(self.mop, QDQ(rb, dt), QTR(f_), QDSP(rb, kk), QDQ(rb, dt))

            g.run(mfma, pre_budget=48)
        e.salu(f"s_add_i32 {SI}, {SI}, 1")
        e.salu(f"s_add_i32 {Q_SN0}, {Q_SN0}, 64")
        e.salu(f"s_xor_b32 {Q_PAR}, {Q_PAR}, 1")
        e.drain_lds()
        if "dq_novm" not in ABL:
            e.raw("s_waitcnt vmcnt(0)")
        if "dq_nobar" not in ABL:
            e.raw("s_barrier")
        e.reset()

    def next_unit_loads(self):
        """The next unit's Q and dO fragments straight into the %[q*] / %[o*] accumulation
        registers (read-write operands; the caller waits before reading them).  Descriptor range
        0 without a next unit."""
        e = self.e
        for what, d in (("q", 68), ("o", 72)):
            e.salu(f"s_mov_b32 s{d}, %[n{what}lo]")
            e.salu(f"s_and_b32 s{d + 1}, %[n{what}hi], 0xffff")
            e.salu(f"s_mov_b32 s{d + 2}, %[n{what}bytes]")
            e.salu(f"s_mov_b32 s{d + 3}, 0x20000")
        for what, d in (("q", 68), ("o", 72)):
            for rb in range(2):
                for ks in range(8):
                    # row block 1: 32 rows further (%[n{what}rs] = 32 row strides, as soffset)
                    so = f"%[n{what}rs]" if rb else "0"
                    e.raw(f"buffer_load_dwordx4 %[{what}{rb * 8 + ks}], %[n{what}o0], s[{d}:{d + 3}], {so} offen offset:{32 * ks}")

    # -- one unit (256 query rows), persistent across units -------------------------------------
    def build(self):
        e = self.e
        e.raw("s_nop 7")
        e.raw("s_nop 7")
        e.salu(f"s_mov_b32 {SM0}, m0")
        for r in range(128):
            e.valu(f"v_accvgpr_write_b32 a{r}, 0", f"a{r}", kind="accw")
        if self.seed:  # -delta blocks (QNDEL): the dP chains' initial accumulators
            for rb in range(2):
                for r in _regs(QNDEL(rb)):
                    e.valu(f"v_sub_f32 {r}, 0, %[del{rb}]", r)
        # DMA cursors: period i requests K(i + 1), V(i + 1); the final period's requests are the
        # next unit's K(0), V(0) (cursors switched to its slices), into the buffer it starts on
        e.salu(f"s_mov_b32 {SKP[0]}, %[klo]")
        e.salu(f"s_mov_b32 {SKP[1]}, %[khi]")
        e.salu(f"s_mov_b32 {SVP[0]}, %[vlo]")
        e.salu(f"s_mov_b32 {SVP[1]}, %[vhi]")
        e.salu(f"s_mov_b32 {SKR}, %[kbytes]")
        e.salu(f"s_mov_b32 {SVR}, %[kbytes]")
        for p0, p1, rem in ((SKP[0], SKP[1], SKR), (SVP[0], SVP[1], SVR)):
            e.salu(f"s_add_u32 {p0}, {p0}, %[tileb]")
            e.salu(f"s_addc_u32 {p1}, {p1}, 0")
            e.salu(f"s_sub_i32 {rem}, {rem}, %[tileb]")
        e.salu(f"s_mov_b32 {SI}, 0")
        e.salu(f"s_mov_b32 {Q_SN0}, 0")
        e.salu(f"s_mov_b32 {Q_PAR}, %[boff]")
        e.salu(f"s_add_i32 {Q_FIN}, %[ntiles], -1")
        e.salu(f"s_min_i32 {Q_NA}, %[na], {Q_FIN}")  # A chain: class A tiles before the final one
        if self.dropout:
            # keep words: tile 0's in %[mw*] (from the previous unit or the caller) -> both sets;
            # period i requests tile i + 1's
            e.salu(f"s_mov_b32 {Q_MOFF[0]}, 256")
            e.salu(f"s_add_u32 {Q_MOFF[1]}, %[mrs], 256")
            e.valu(f"v_mov_b32 {QMO}, %[mo0]", QMO)
            for rb in range(2):
                for h in range(2):
                    for st in range(2):
                        e.valu(f"v_mov_b32 {QMW(st, rb, h)}, %[mw{2 * rb + h}]", QMW(st, rb, h))
        # this unit's K(0), V(0) (requested by the previous unit or before the statement), Q, dO
        e.raw("s_waitcnt vmcnt(0) lgkmcnt(0)")
        e.raw("s_barrier")
        e.reset()
        e.raw(f"s_cmp_lt_i32 {Q_FIN}, 0")
        e.raw("s_cbranch_scc0 .Lhp%=_loop")
        # no tile: the next unit's K(0), V(0) into buffer boff as a DMA-only period of parity 1-boff
        self.switch_cursors()
        e.salu(f"s_xor_b32 {Q_PAR}, {Q_PAR}, 1")
        e.raw(f"s_cmp_eq_u32 {Q_PAR}, 0")
        e.raw("s_cbranch_scc1 .Lhp%=_D0")
        e.raw("s_branch .Lhp%=_D1")
        e.raw(".balignl 64, 0xbf800000", 0)
        e.label(".Lhp%=_loop")
        e.raw(f"s_cmp_gt_i32 {SI}, {Q_FIN}")
        e.raw("s_cbranch_scc1 .Lhp%=_end")
        e.raw(f"s_cmp_eq_u32 {SI}, {Q_FIN}")
        e.raw("s_cbranch_scc0 .Lhp%=_cls")
        self.switch_cursors()
        e.label(".Lhp%=_cls")
        e.raw(f"s_cmp_lt_i32 {SI}, %[na]")
        e.raw("s_cbranch_scc1 .Lhp%=_clsA")
        e.raw(f"s_cmp_le_i32 {SI}, %[last]")
        e.raw("s_cbranch_scc1 .Lhp%=_clsB")
        e.raw(f"s_cmp_eq_u32 {Q_PAR}, 0")
        e.raw("s_cbranch_scc1 .Lhp%=_D0")
        e.raw("s_branch .Lhp%=_D1")
        # class A runs as a chain (the final tile excluded: its cursors switch first)
        e.label(".Lhp%=_clsA")
        e.raw(f"s_cmp_eq_u32 {SI}, {Q_FIN}")
        e.raw("s_cbranch_scc1 .Lhp%=_A1f")
        e.raw(f"s_cmp_eq_u32 {Q_PAR}, 0")
        e.raw("s_cbranch_scc0 .Lhp%=_A1")
        e.label(".Lhp%=_A0")
        self.period(0, "A")
        e.raw(f"s_cmp_ge_i32 {SI}, {Q_NA}")
        e.raw("s_cbranch_scc1 .Lhp%=_loop")
        e.label(".Lhp%=_A1")
        self.period(1, "A")
        e.raw(f"s_cmp_lt_i32 {SI}, {Q_NA}")
        e.raw("s_cbranch_scc1 .Lhp%=_A0")
        e.raw("s_branch .Lhp%=_loop")
        e.label(".Lhp%=_A1f")  # the final tile, class A: parity dispatch
        e.raw(f"s_cmp_eq_u32 {Q_PAR}, 0")
        e.raw("s_cbranch_scc1 .Lhp%=_A0")
        e.raw("s_branch .Lhp%=_A1")
        e.label(".Lhp%=_clsB")
        e.raw(f"s_cmp_eq_u32 {Q_PAR}, 0")
        e.raw("s_cbranch_scc0 .Lhp%=_B1")
        for par in (0, 1):
            e.label(f".Lhp%=_B{par}")
            self.period(par, "B")
            e.raw("s_branch .Lhp%=_loop")
        for par in (0, 1):
            e.label(f".Lhp%=_D{par}")
            self.period(par, "D")
            e.raw("s_branch .Lhp%=_loop")
        e.label(".Lhp%=_end")
        if self.dropout:
            # the final period requested the next unit's tile-0 words into set Q_PAR (flipped since)
            e.raw(f"s_cmp_eq_u32 {Q_PAR}, 0")
            e.raw("s_cbranch_scc0 .Lhp%=_mw1")
            for st in range(2):
                if st == 1:
                    e.label(".Lhp%=_mw1")
                for rb in range(2):
                    for h in range(2):
                        e.raw(f"v_mov_b32 %[mw{2 * rb + h}], {QMW(st, rb, h)}")
                if st == 0:
                    e.raw("s_branch .Lhp%=_mwd")
            e.label(".Lhp%=_mwd")
        else:
            # the next unit's Q / dO straight into the operand registers, left in flight across the
            # epilogue (the dropout variant loads them in its own statement after the epilogue:
            # gen_dq_load_next, nothing in flight between statements)
            self.next_unit_loads()
        e.drain_lds()
        e.salu(f"s_mov_b32 m0, {SM0}")
        e.raw("s_nop 15")
        e.raw("s_nop 15")
        return e.out

    def switch_cursors(self):
        e = self.e
        e.salu(f"s_mov_b32 {SKP[0]}, %[nklo]")
        e.salu(f"s_mov_b32 {SKP[1]}, %[nkhi]")
        e.salu(f"s_mov_b32 {SVP[0]}, %[nvlo]")
        e.salu(f"s_mov_b32 {SVP[1]}, %[nvhi]")
        e.salu(f"s_mov_b32 {SKR}, %[nkbytes]")
        e.salu(f"s_mov_b32 {SVR}, %[nkbytes]")
        if self.dropout:  # the final period's keep words: the next unit's tile 0
            e.valu(f"v_mov_b32 {QMO}, %[nmo0]", QMO)
            e.salu(f"s_mov_b32 {Q_MOFF[0]}, 0")
            e.salu(f"s_mov_b32 {Q_MOFF[1]}, %[mrs]")


def gen_dq_function(bf16, causal, dropout=False):
    g = DqGen(bf16, causal, dropout)
    lines = g.build()
    name = f"dq_hp_main_{'bf16' if bf16 else 'f16'}_{'causal' if causal else 'full'}{'_drop' if dropout else ''}"
    nv = DQ_NVGPR_DROP if dropout else DQ_NVGPR + 32
    clob = [f'"v{i}"' for i in range(nv)] + [f'"a{i}"' for i in range(128)] + \
           [f'"s{i}"' for i in _sgprs_used(lines)] + ['"vcc"', '"scc"', '"memory"']
    qops = ", ".join(f'[q{i}] "+a"(q[{i}])' for i in range(16))
    oops = ", ".join(f'[o{i}] "+a"(o[{i}])' for i in range(16))
    mops = (",\n        " + ", ".join(f'[mw{i}] "+v"(mw[{i}])' for i in range(4))) if dropout else ""
    nxt_v = [] if dropout else ["nqo0", "noo0"]
    nxt_s = [] if dropout else ["nqlo", "nqhi", "nqbytes", "nolo", "nohi", "nobytes", "nqrs", "nors"]
    vops = ["kb0", "kb1", "ta", "tb", "off0", "off1", "off2", "off3", "rel0", "rel1", "lse0", "lse1", "del0", "del1"] + \
        nxt_v + (["mo0", "nmo0", "msh"] if dropout else [])
    sops = ["na", "last", "ntiles", "tileb", "kbytes", "mlds", "klo", "khi", "vlo", "vhi", "sc",
            "boff", "nklo", "nkhi", "nvlo", "nvhi", "nkbytes"] + nxt_s + (["mdesc", "mrs", "dsc"] if dropout else [])
    marg = ", uint32_t (&mw)[4]" if dropout else ""
    inout = ("this unit's Q and dO fragments in (the next unit's: gen_dq_load_next)" if dropout else
             "this unit's Q and dO fragments in, the NEXT unit's out -- still in flight (wait before\n// reading them)")
    src = f"""// hand-placed dQ unit ({'bf16' if bf16 else 'fp16'}, {'causal' if causal else 'non-causal'}{', dropout' if dropout else ''}): {len(lines)} lines, {g.e.n_mfma} MFMAs
// q / o: {inout}{'; mw: the keep words of tile 0, in and (next unit) out' if dropout else ''}
FA2_DEV void {name}(u32x4 (&q)[16], u32x4 (&o)[16], const DqHpArgs& a{marg}) {{
  asm volatile(
{_asm_body(lines)}
      : {qops},
        {oops}{mops}
      : {", ".join(f'[{n}] "v"(a.{n})' for n in vops)},
        {", ".join(f'[{n}] "s"(a.{n})' for n in sops)}
      : {", ".join(clob)});
}}
"""
    return src


def _asm_body(lines):
    return "\n".join(f'      "{l}\\n"' for l in lines)


def _sgprs_used(lines):
    """The fixed SGPRs a statement names (its clobbers: no more than it uses, so the compiler
    keeps the rest for the values live across it)."""
    used = set()
    for l in lines:
        for m in re.finditer(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b", l):
            if m.group(3):
                used.add(int(m.group(3)))
            else:
                used.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return sorted(used)


def gen_dq_load_next():
    """The dropout dQ's next-unit Q / dO fragments: loads and their wait in ONE statement (outputs
    early-clobber), so no load is in flight while compiler code runs (the compiler
    moved in-flight "+a" operands of the spilling dropout variant and read them early)."""
    g = DqGen(True, False, False)
    g.next_unit_loads()
    # s_nop 12: marker of tests/test_code_objects.py (end of the in-flight window: none here)
    lines = ["s_nop 12"] + g.e.out + ["s_waitcnt vmcnt(0)"]
    qops = ", ".join(f'[q{i}] "=&a"(q[{i}])' for i in range(16))
    oops = ", ".join(f'[o{i}] "=&a"(o[{i}])' for i in range(16))
    ins = ", ".join([f'[{n}] "v"(a.{n})' for n in ("nqo0", "noo0")] +
                    [f'[{n}] "s"(a.{n})' for n in ("nqlo", "nqhi", "nqbytes", "nolo", "nohi", "nobytes", "nqrs", "nors")])
    clob = ", ".join([f'"s{i}"' for i in _sgprs_used(lines)] + ['"memory"'])
    return f"""// the next unit's Q / dO fragments (dropout dQ), loaded and waited for in one statement
FA2_DEV void dq_hp_load_next(u32x4 (&q)[16], u32x4 (&o)[16], const DqHpArgs& a) {{
  asm volatile(
{_asm_body(lines)}
      : {qops},
        {oops}
      : {ins}
      : {clob});
}}
"""


def gen_fwd_function(bf16, causal, exact=True, dt=128, dropout=False):
    out = []
    nq = 2 * (dt // 16)  # Q fragments (two row blocks x k-steps)
    for stamp in ((False,) if dropout else (False, True)):
        g = FwdGen(bf16, causal, exact, stamp, dt, dropout)
        lines = g.build()
        name = f"fwd_hp_main_{'bf16' if bf16 else 'f16'}_{'causal' if causal else 'full'}{'' if exact else '_ps'}" + \
            ("" if dt == 128 else f"_d{dt}") + ("_drop" if dropout else "")
        # O^T a[0 : dt], K / V^T rings a[192:223]; every AGPR but the Q operands' (a[128:191] at
        # D = 128, a[64:95] at D = 64) clobbered, so the compiler has no room to move them
        acc = list(range(0, dt)) + list(range(dt + 2 * dt // 4 if dt == 64 else 192, 256))
        clob = [f'"v{i}"' for i in range(N_VGPR)] + [f'"a{i}"' for i in acc] + \
               [f'"s{i}"' for i in _sgprs_used(lines)] + ['"vcc"', '"scc"', '"memory"']
        qops = ", ".join(f'[q{i}] "+a"(q[{i}])' for i in range(nq))
        stops = ", " + ", ".join(f'[st{i}] "=&s"(st[{i}])' for i in range(4)) if stamp else ""
        starg = ", uint32_t (&st)[4]" if stamp else ""
        dops = ('\n        [mvo0] "v"(a.mvo[0]), [mvo1] "v"(a.mvo[1]), [hh4] "v"(a.hh4), [mlo] "s"(a.mlo), '
                '[mhi] "s"(a.mhi), [mbytes] "s"(a.mbytes),' if dropout else "")
        out.append(f"""{'#if FA2_HP_STAMPS' if stamp else '#if !FA2_HP_STAMPS'}
// hand-placed unit ({'bf16' if bf16 else 'fp16'}, {'causal' if causal else 'non-causal'}, {'exact scale' if exact else 'pre-scaled Q'}{', dropout' if dropout else ''}{', stamped' if stamp else ''}): {len(lines)} lines, {g.e.n_mfma} MFMAs
// q: this unit's Q fragments in, the NEXT unit's Q fragments out -- still in flight (the next
// statement waits for them first; nothing may read q in between)
FA2_DEV void {name}(u32x4 (&q)[{nq}], const FwdHpArgs& a, float (&m_out)[2], float (&l_out)[2]{starg}) {{
  asm volatile(
{_asm_body(lines)}
      : [mo0] "=&v"(m_out[0]), [mo1] "=&v"(m_out[1]), [lo0] "=&v"(l_out[0]), [lo1] "=&v"(l_out[1]), {qops}{stops}
      : [kb0] "v"(a.kb0), [kb1] "v"(a.kb1), [va] "v"(a.va), [vb] "v"(a.vb),{dops}
        {", ".join(f'[off{i}] "v"(a.off[{i}])' for i in range(dt // 32))},
        [rel0] "v"(a.rel[0]), [rel1] "v"(a.rel[1]), [nqo0] "v"(a.nqo[0]), [nqo1] "v"(a.nqo[1]),
        [na] "s"(a.na), [last] "s"(a.last), [ntiles] "s"(a.ntiles), [mask0] "s"(a.mask0),
        [tileb] "s"(a.tileb), [kbytes] "s"(a.kbytes), [mlds] "s"(a.mlds),
        [klo] "s"(a.klo), [khi] "s"(a.khi), [vlo] "s"(a.vlo), [vhi] "s"(a.vhi), [uz] "s"(a.uz),
        [boff] "s"(a.boff), [nklo] "s"(a.nklo), [nkhi] "s"(a.nkhi), [nvlo] "s"(a.nvlo), [nvhi] "s"(a.nvhi),
        [nkbytes] "s"(a.nkbytes), [nqlo] "s"(a.nqlo), [nqhi] "s"(a.nqhi), [nqbytes] "s"(a.nqbytes)
      : {", ".join(clob)});
}}
#endif
""")
    return "".join(out)


# Each read statement clobbers every accumulator register: a value live across them (the next
# unit's Q / dO fragments, "+a" operands of the main statement) then cannot be placed in
# a[0:127] anywhere between the main statement and the last read -- the compiler moving one
# there early would overwrite accumulators not read yet (tests/test_code_objects.py checks the ISA).
ACC_CLOBBER = ", ".join(f'"a{i}"' for i in range(128))


def gen_read_o(ndt=4):
    n = 32 * ndt
    clob = ", ".join(f'"a{i}"' for i in range(n))
    parts = [f"// O^T accumulators a[0:{n - 1}] -> registers (after the main statement's final drain)",
             f"FA2_DEV void fwd_hp_read_o{'' if ndt == 4 else f'_d{32 * ndt}'}(f32x16 (&o)[2][{ndt}]) {{"]
    for rb in range(2):
        for dt in range(ndt):
            base = (rb * ndt + dt) * 16
            outs = ", ".join(f'"=v"(o[{rb}][{dt}][{i}])' for i in range(16))
            body = "".join(f"v_accvgpr_read_b32 %{i}, a{base + i}\\n" for i in range(16))
            parts.append(f'  asm volatile("{body}" : {outs} : : {clob});')
    parts.append("}")
    return "\n".join(parts) + "\n"


def write_headers():
    os.makedirs(GEN, exist_ok=True)
    out = ["// generated by fa2_triton_amd/hp_gen.py -- do not edit", "#pragma once", "", "namespace fa2 {", ""]
    for bf16 in (True, False):
        for causal in (True, False):
            for exact in (True, False):
                out.append(gen_fwd_function(bf16, causal, exact))
            out.append(gen_fwd_function(bf16, causal, True, dropout=True))
            # (FwdGen(dt=64) builds a D = 64 unit too; measured no faster than fwd_pipe_kernel at
            # D = 64, where the softmax VALU bounds both -- DESIGN.md section 6 -- so not emitted)
    out.append(gen_read_o())
    out.append("}  // namespace fa2\n")
    text = "\n".join(out)
    paths = [_write(os.path.join(GEN, "fwd_hp_body.h"), text)]
    out = ["// generated by fa2_triton_amd/hp_gen.py -- do not edit", "#pragma once", "", "namespace fa2 {", ""]
    for bf16 in (True, False):
        for causal in (True, False):
            for dropout in (False, True):
                out.append(gen_dkdv_function(bf16, causal, dropout))
    out.append(gen_read_dkdv())
    out.append("// LDS layout of the dK/dV statements (DkdvGen, DkLayout): step buffers, V rows at v0, LSE2 /\n"
               "// -delta rows at rows, the dropout keep words at words; size in bytes\n"
               "template <bool DROPOUT> struct DkdvLds;")
    for dropout in (False, True):
        L = DkLayout(DK_NBUF_DROP if dropout else DK_NBUF_PLAIN)
        out.append(f"template <> struct DkdvLds<{'true' if dropout else 'false'}> {{\n"
                   f"  static constexpr int nbuf = {L.nbuf}, v0 = {L.v0}, rows = {L.rows}, words = {L.w0}, "
                   f"size = {L.lds_drop if dropout else L.lds};\n}};")
    out.append("")
    out.append("}  // namespace fa2\n")
    paths.append(_write(os.path.join(GEN, "dkdv_hp_body.h"), "\n".join(out)))
    out = ["// generated by fa2_triton_amd/hp_gen.py -- do not edit", "#pragma once", "", "namespace fa2 {", ""]
    for bf16 in (True, False):
        for causal in (True, False):
            for dropout in (False, True):
                out.append(gen_dq_function(bf16, causal, dropout))
    out.append(gen_dq_load_next())
    out.append(gen_read_o().replace("fwd_hp_read_o", "dq_hp_read").replace("O^T accumulators", "dQ^T accumulators"))
    out.append("}  // namespace fa2\n")
    paths.append(_write(os.path.join(GEN, "dq_hp_body.h"), "\n".join(out)))
    return paths


def _write(path, text):
    if not os.path.exists(path) or open(path).read() != text:
        with open(path, "w") as f:
            f.write(text)
    return path


if __name__ == "__main__":
    print(write_headers())
