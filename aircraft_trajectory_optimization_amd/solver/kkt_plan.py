'''
Static plan of the batched on-device KKT factorisation (include/ato_kkt.h).

The KKT matrix of the raceline interior-point step (IPOPT's augmented system; the reference
factorises it with MUMPS / MA97 inside ca.nlpsol, base_raceline.py:752-799)

    K = [ W + diag_x   J^T    ]     n variables, m constraint rows, dim = n + m
        [ J            diag_r ]

is ordered by interval (stage) exactly as solver/kkt_blocks.py does on the host: every variable
belongs to the interval it lives in, a row touching one stage or two neighbouring stages joins
the later one, and rows reaching further (loop closure, equal step sizes) form the border.

For every stage s the device works on an AUGMENTED block of positions

    own(s)            the stage's variables, then its rows          (eligible pivots)
    coupling(s+1)     rows of stage s+1 with entries on stage-s variables
    border            all border rows

The own positions are eliminated with Bunch-Kaufman pivoting restricted to own(s); what is left
in the trailing (coupling + border) block is the Schur complement, which is CARRIED into stage
s+1 (coupling positions are own positions there, border positions stay border). After the last
stage a pseudo-stage holds the border alone and is factorised completely. The inertia of K is the
sum of the inertias of all pivots (Haynsworth), which is what IPOPT's inertia correction needs.

This module builds, once per problem structure, the integer tables the kernels read:
position -> KKT index, the lower-triangle entry list of every augmented block grouped by
32-row strip with the source of each value (Hessian entry, Jacobian entry, variable or row
diagonal), the carry map, and the per-stage storage offsets of the factor.
'''
from dataclasses import dataclass
from typing import List

import numpy as np

SRC_H, SRC_J, SRC_DX, SRC_DR = 0, 1, 2, 3
SRC_SHIFT = 29
TILE = 32
MAX_TILES = 8              # augmented blocks up to 256 positions (kernel register tiles)


def src_code(kind: int, idx: int) -> int:
    return (kind << SRC_SHIFT) | int(idx)


@dataclass
class KKTPlan:
    n: int                      # variables
    m: int                      # rows
    dim: int                    # n + m
    n_stages: int               # intervals + 1 border pseudo-stage
    tiles: int                  # 32-wide tiles of the largest augmented block
    stage_ptr: np.ndarray       # [S+1] into pos_index
    n_own: np.ndarray           # [S]
    pos_index: np.ndarray       # [P] KKT index of every augmented position
    carry_dst: np.ndarray       # [P] trailing position -> position in the next stage (-1: own)
    ent_ptr: np.ndarray         # [S * tiles + 1] entries of (stage, strip)
    ent_pos: np.ndarray         # [E] (pa << 16) | pb with pa >= pb
    ent_src: np.ndarray         # [E, 2] source codes (-1: none)
    l_off: np.ndarray           # [S] offset of the stage's factor columns (doubles, per instance)
    l_size: int                 # doubles of factor columns per instance
    piv_off: np.ndarray         # [S] offset of the stage's pivot records (per instance)
    block_sizes: np.ndarray     # [S] augmented size

    @property
    def max_block(self) -> int:
        return int(self.block_sizes.max())


def row_stages(n, m, var_stage, j_row_ptr, j_col) -> np.ndarray:
    ''' stage of every row: the later stage of a row touching one or two neighbouring stages,
    -1 for border rows (same rule as solver/kkt_blocks.BlockKKT) '''
    var_stage = np.asarray(var_stage)
    cnt = np.diff(np.asarray(j_row_ptr))
    jr = np.repeat(np.arange(m), cnt)
    st = var_stage[np.asarray(j_col)]
    lo = np.full(m, np.iinfo(np.int64).max)
    hi = np.full(m, -1)
    np.minimum.at(lo, jr, st)
    np.maximum.at(hi, jr, st)
    rs = np.where(hi - lo <= 1, hi, -1)
    rs[hi < 0] = 0
    return rs


def build_plan(n: int, m: int, var_stage, j_row_ptr, j_col, h_row_ptr, h_col) -> KKTPlan:
    var_stage = np.asarray(var_stage, np.int64)
    j_row_ptr = np.asarray(j_row_ptr, np.int64)
    j_col = np.asarray(j_col, np.int64)
    h_row_ptr = np.asarray(h_row_ptr, np.int64)
    h_col = np.asarray(h_col, np.int64)
    S = int(var_stage.max()) + 1
    rs = row_stages(n, m, var_stage, j_row_ptr, j_col)
    jr = np.repeat(np.arange(m), np.diff(j_row_ptr))
    hr = np.repeat(np.arange(n), np.diff(h_row_ptr))
    if len(hr) and np.any(var_stage[hr] != var_stage[h_col]):
        raise ValueError('Hessian couples different stages; the staged KKT does not apply')

    border = n + np.nonzero(rs < 0)[0]
    own: List[np.ndarray] = []
    for s in range(S):
        own.append(np.concatenate([np.nonzero(var_stage == s)[0], n + np.nonzero(rs == s)[0]]))
    # coupling(s+1): rows of stage s+1 with entries on stage-s variables
    cpl_rows = (rs[jr] >= 1) & (var_stage[j_col] == rs[jr] - 1)
    coupling = [np.zeros(0, np.int64) for _ in range(S + 1)]
    for s in range(1, S):
        coupling[s] = n + np.unique(jr[cpl_rows & (rs[jr] == s)])

    blocks = []                 # augmented position lists (KKT indices)
    n_own = []
    for s in range(S):
        blocks.append(np.concatenate([own[s], coupling[s + 1] if s + 1 < S else np.zeros(0, np.int64), border]))
        n_own.append(len(own[s]))
    blocks.append(border.copy())
    n_own.append(len(border))
    NS = S + 1
    sizes = np.array([len(b) for b in blocks])
    tiles = int(max(1, -(-sizes.max() // TILE)))
    if tiles > MAX_TILES:
        raise ValueError(f'augmented KKT block of {sizes.max()} positions exceeds the device limit '
                         f'{MAX_TILES * TILE}')
    pos_of = []                 # KKT index -> position, per stage
    for b in blocks:
        d = np.full(n + m, -1, np.int64)
        d[b] = np.arange(len(b))
        pos_of.append(d)

    # ---- entries: (stage, pa, pb, src1, src2)
    ent = {s: {} for s in range(NS)}

    def add(s, i, j, code):
        pa, pb = pos_of[s][i], pos_of[s][j]
        assert pa >= 0 and pb >= 0, (s, i, j)
        if pa < pb:
            pa, pb = pb, pa
        key = (int(pa), int(pb))
        lst = ent[s].setdefault(key, [])
        lst.append(code)

    for e in range(len(h_col)):             # Hessian (lower, same stage)
        r, c = int(hr[e]), int(h_col[e])
        add(int(var_stage[r]), r, c, src_code(SRC_H, e))
    for j in range(n):                       # variable diagonal
        add(int(var_stage[j]), j, j, src_code(SRC_DX, j))
    for e in range(len(j_col)):              # Jacobian (row i, variable j): stage of the variable
        i, j = int(jr[e]), int(j_col[e])
        add(int(var_stage[j]), n + i, j, src_code(SRC_J, e))
    for i in range(m):                       # row diagonal
        s = int(rs[i]) if rs[i] >= 0 else S
        add(s, n + i, n + i, src_code(SRC_DR, i))

    ent_ptr = [0]
    ent_pos, ent_src = [], []
    for s in range(NS):
        keys = sorted(ent[s].keys(), key=lambda k: (k[0] // TILE, k[0], k[1]))
        strips = [[] for _ in range(tiles)]
        for k in keys:
            srcs = ent[s][k]
            if len(srcs) > 2:
                raise ValueError(f'KKT entry {k} of stage {s} has {len(srcs)} sources')
            strips[k[0] // TILE].append((k, srcs))
        for I in range(tiles):
            for (pa, pb), srcs in strips[I]:
                ent_pos.append((pa << 16) | pb)
                ent_src.append([srcs[0], srcs[1] if len(srcs) > 1 else -1])
            ent_ptr.append(len(ent_pos))

    # ---- carry map: trailing position of stage s -> position in stage s+1
    stage_ptr = np.concatenate([[0], np.cumsum(sizes)])
    carry_dst = np.full(int(stage_ptr[-1]), -1, np.int64)
    for s in range(NS - 1):
        b = blocks[s]
        for q in range(n_own[s], len(b)):
            dst = pos_of[s + 1][b[q]]
            assert dst >= 0
            carry_dst[stage_ptr[s] + q] = dst

    # ---- factor storage: compact columns of live positions after each step
    l_off, piv_off = [], []
    lo = po = 0
    for s in range(NS):
        A, o = int(sizes[s]), int(n_own[s])
        l_off.append(lo)
        piv_off.append(po)
        lo += o * A - o * (o + 1) // 2
        po += o
    return KKTPlan(n=n, m=m, dim=n + m, n_stages=NS, tiles=tiles,
                   stage_ptr=stage_ptr.astype(np.int32), n_own=np.asarray(n_own, np.int32),
                   pos_index=np.concatenate(blocks).astype(np.int32), carry_dst=carry_dst.astype(np.int32),
                   ent_ptr=np.asarray(ent_ptr, np.int32), ent_pos=np.asarray(ent_pos, np.int32),
                   ent_src=np.asarray(ent_src, np.int32).reshape(-1, 2), l_off=np.asarray(l_off, np.int64),
                   l_size=int(lo), piv_off=np.asarray(piv_off, np.int32), block_sizes=sizes.astype(np.int32))
