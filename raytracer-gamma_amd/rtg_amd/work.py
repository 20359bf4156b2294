"""Executed-work model of the trace kernel (the roofline's work).

The counting build of the default kernel (launch variant 120, rtg_diag_counts)
counts, per WAVE, how often each code unit of the traversal executes (a unit
that any lane of a wave executes costs that wave the unit's instructions: the
SIMD issues them for all 64 lanes).  `UNIT_COST` is the unit's VALU issue cost
in wave-instruction slots — the vector arithmetic, compare and select
operations of the unit's source in rtg_trace.h as CDNA4 executes them (a
transcendental v_sqrt / v_rcp / v_rsq or an f64 operation counts 2 slots, the
correctly rounded float division 10, sqrt_rn 12 = v_sqrt + 2 neighbour steps +
range check, rcp_fast 4, rcp_sqrt_rn 16, the Markstein quotient 5).  Scalar
work (loop control, scalar record loads, wave-uniform masks) and memory
instructions are not counted: they issue on other units.

    executed VALU lane-ops = 64 * sum_u waves_u * UNIT_COST[u]
    roofline.achieved      = that / kernel time;  peak 78.6 T (VALU_PEAK_TOPS)

The model is checked against the PMC count of issued VALU instructions
(SQ_INSTS_VALU, tools/gpu_pmc.sh) of the same frame: bench.py reports the
ratio.  Unit names follow rtg_amd.UNIT_NAMES (rtg_trace.h kU* slots).
"""
from __future__ import annotations

# VALU slots per wave-level execution of each unit (see the module docstring).
UNIT_COST = {
    # make_query: a = d.d (5), 4a, 2a, a(1-K), a(1-K_B) (4), range test (3),
    # 1/2a = rcp_fast (4)
    "U.query": 16,
    # closest_hit_sel_fused: bp = 2 d.c (6), bp^2 - 4a oc (3), >= 0 (1)
    "U.primIter": 10,
    # its root test: sqrt_rn (12), two quotients (2 x (1 + 5)), accept tests and
    # selects (8), closest update (4)
    "U.primExact": 36,
    # pass1_rad (3 sub, 3 + 3 fused dot terms, 2 fma) + sign test
    "U.selIter": 12,
    # ray_sphere_k: p (3), b (6), cc (6), radicand (3), test (1), sqrt_rn (12),
    # quotients (12), accept (8); closest update (4)
    "U.selExact": 55,
    # pass1_rad + sign test + not-yet-blocked
    "U.shdIter": 13,
    # ray_sphere_k (51) + t < 1000, |t D|^2 < gap (3 + 5 + 2), blocked select (1)
    "U.shdExact": 62,
    # sphere h's ray_sphere_k (51), exit point (9), two guard tests (10 + 7)
    "U.enterHead": 77,
    # the lane's own-mask bit test
    "U.enterIter": 3,
    # ray_sphere_k (51) + lexicographic (t, index) update (7)
    "U.enterExact": 58,
    # candidate_mask: 4 x (pass1_rad 11 + sign shift 1)
    "U.fullGroup": 48,
    # ray_sphere with the per-quotient range select (55) + update (4)
    "U.fullExact": 59,
    # node pop and front-to-back push are scalar; the ballots' compares
    "U.bvhNode": 2,
    # p (3), x (3), |p|^2 (3), distance prune (5), bound / sphere screen (4),
    # lane predicates (2)
    "U.bvhSlot": 20,
    # ray_sphere (55) + (t, index) update or blocking test (5)
    "U.bvhExact": 60,
    # |pt - c|^2 <= cr (9), first-found update (4)
    "U.contIter": 13,
    # 4 x 9 + bit assembly (4) + lowest-bit update (3)
    "U.cont4": 43,
    # 4 x 9 + 4 x min update (3)
    "U.contBvhNode": 48,
    # |d|^2 (5), rsq (2), d / |d| (3), cos to the bundle axis (5), tiers (2)
    "U.cone": 17,
    # readlane + compare + own-mask select
    "U.maskIter": 4,
    # node dispatch tests (entered / origin-ball / hit / significant I)
    "U.node": 12,
    # P (6), N = vnorm(P - c) (3 + 5 + 16 + 3), guard test (9), opacity terms and
    # colour (13)
    "U.shade": 55,
    # L - P (3), facing-away pre-test: N.dist (3), sum |N_k dist_k| (3), tests (3)
    "U.light": 12,
    # gap (5), rcp_sqrt_rn (16), dir (3), incidence (5), test (1)
    "U.lightDir": 30,
    # mask-union predicates of the shadow ray
    "U.shadow": 3,
    # incidence / gap (10), sum += intensity * Lcol (6)
    "U.lit": 16,
    # cos (5), clamps (4), f64 sinA1 (37), test point (6), |D| test (7), n ratio
    # (10), solveQuadratic incl. sqrt_rn (28), the two candidate directions (32),
    # cosA2 (16), two f64 Fresnel factors (80), R (2), reflection colour (18)
    "U.refr": 245,
    # the same without the refracted direction (solveQuadratic and candidates)
    "U.refrLeaf": 185,
    # 2 d.N (6), d - p N (6), vnorm (27), origin P + 0.01 rd (6), flags (3)
    "U.push": 48,
    # frame metadata (6), entering / origin-ball tests (8), child I (7), moves (7)
    "U.descend": 28,
    # colour sum (3), stage tests and frame update (9)
    "U.unwind": 12,
    # sphere-list queries of BVH scenes (blocked_cap; closest_enter_list /
    # container_list): one record's pass-1 screen (+ not-blocked) or containment test
    "U.capIter": 13,
    "U.ovIter": 13,
    # lane -> pixel / sample (6), sample_dir + vnorm (38), scaled sum, ordered
    # pixel sums (3 + 27), NaN canonicalisation and row bookkeeping (6)
    "U.sample": 80,
    # a wave's prologue (frame pointers, group index, the next launch's
    # counters), its list walk and exit: also every wave past the listed groups
    "U.wave": 20,
}

# The unit prices above are the SOURCE prices; the bench line uses prices
# fitted to the hardware's SQ_INSTS_VALU (tools/calib_units.py) over 29 scenes
# of both kernel kinds on the final round-6 sources: the bench configs C1-C5
# (C4 at half and C5 at a quarter of each side) weighted 10x, 14 seeded masked
# and 10 seeded BVH scenes; least squares on the relative residuals with a
# ridge toward the source prices and bounds of 0.6-1.7x the SOURCE prices
# (never an earlier fit's, so refits do not drift: ADVICE r05).  rms model/PMC
# error over the set: source prices 10.4 %, fitted 2.7 % (in sample).
# Held out, each bench config left out of its own fit: c2 0.992, c3 1.011, c4 0.982, c5 1.010;
# a fit on the seeded scenes alone: c2 1.009, c3 1.016, c4 0.993, c5 1.013 (FIT_RECORD).
FIT_RECORD = "profiles/r06/calib_units/fit.json"
UNIT_COST_SOURCE = dict(UNIT_COST)
UNIT_COST.update({
    "U.query": 19.97,
    "U.primIter": 11.58,
    "U.primExact": 48.38,
    "U.selIter": 11.43,
    "U.selExact": 55.98,
    "U.shdIter": 13.54,
    "U.shdExact": 57.52,
    "U.enterHead": 81.57,
    "U.enterIter": 2.97,
    "U.enterExact": 39.09,
    "U.fullGroup": 50.98,
    "U.fullExact": 81.25,
    "U.bvhNode": 2.0,
    "U.bvhSlot": 20.39,
    "U.bvhExact": 59.4,
    "U.contIter": 12.8,
    "U.contBvhNode": 47.32,
    "U.cone": 16.8,
    "U.maskIter": 4.02,
    "U.node": 13.37,
    "U.shade": 81.94,
    "U.light": 12.84,
    "U.lightDir": 35.96,
    "U.shadow": 3.06,
    "U.lit": 17.88,
    "U.refr": 216.57,
    "U.refrLeaf": 270.71,
    "U.push": 50.08,
    "U.descend": 27.69,
    "U.unwind": 11.92,
    "U.capIter": 10.3,
    "U.ovIter": 11.19,
    "U.sample": 136.0,
    "U.wave": 26.08,
})

VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # one wave64 VALU op per 2 cycles per SIMD


def executed_work(names, waves, lanes=None):
    """Executed VALU work from the counting build's per-unit counters.
    Returns {"valu_slots": wave-instruction slots, "lane_ops": x 64,
    "units": {name: {"waves", "lanes", "slots"}}} over the kU* units."""
    units = {}
    slots = 0
    for k, nm in enumerate(names):
        if nm not in UNIT_COST:
            continue
        w = int(waves[k])
        s = w * UNIT_COST[nm]
        slots += s
        units[nm] = {"waves": w, "slots": s}
        if lanes is not None:
            units[nm]["lanes"] = int(lanes[k])
            units[nm]["lane_util"] = round(int(lanes[k]) / (64.0 * w), 3) if w else None
    return {"valu_slots": slots, "lane_ops": 64 * slots, "units": units}
