'''
Static plan of the batched on-device KKT factorisation (include/ato_kkt.h).

The KKT matrix of the raceline interior-point step (IPOPT's augmented system; the reference
factorises it with MUMPS / MA97 inside ca.nlpsol, base_raceline.py:752-799)

    K = [ W + diag_x   J^T    ]     n variables, m constraint rows, dim = n + m
        [ J            diag_r ]

is factorised by a MULTIFRONTAL symmetric-indefinite LDL^T over an elimination tree of
FRONTS. A front owns a set of KKT indices (its eliminated, "own" positions, listed first) and
has a trailing set (positions that its own rows touch and that are eliminated later, by its
ancestors). The device assembles the front's dense block from the original entries assigned
to it plus the contribution blocks of its children (extend-add), eliminates the own positions
with Bunch-Kaufman pivoting restricted to them, and leaves the Schur complement of the
trailing block as the front's contribution to its parent. Fronts of one LEVEL are independent
(their children are all in lower levels), so a level is one launch over (front, instance)
pairs. The inertia of K is the sum of the inertias of all pivots (Haynsworth) -- exactly what
IPOPT's inertia correction needs.

Orderings of the interval chain (every variable belongs to one interval, the Hessian is block
diagonal by interval, almost every row touches one interval or two neighbouring ones):

  'nd'     nested dissection (default). The separator of boundary j (between intervals j-1
           and j) holds the LINK rows touching both intervals (continuity) and the ANCHOR
           variables of interval j they touch (the new interval's first node). The leaves are
           the interval interiors (all other variables of the interval and the rows touching
           only it): independent fronts, all eliminated in parallel; the anchors pin nothing
           inside a leaf, so the collocation defects there determine the later nodes and the
           leaf blocks stay non-singular (interior rows that touch only anchors join the
           separator). Separators are joined by recursive bisection, the
           border rows (loop closure: rows spanning non-neighbouring intervals) form the root;
           HUB variables (a global gate phase's first step size, tied to every step of the phase
           by the equal-step rows) are eliminated at the root and left out of the row spans, so
           those rows stay inside their intervals. The critical path of one factorisation is one leaf plus
           log2(N) separators instead of the whole chain. Variable / row pairs isolated inside an
           interval (the input rates and their defect rows) form a child front of the leaf
           (split_pairs), which shrinks the leaf block. With `saddle` pairs (collocation_saddle:
           the states of nodes 1..K of an interval and their ODE defect rows) a second child front
           of the leaf holds the saddle block [[H_XX, J_YX^T], [J_YX, 0]]; J_YX is square and (for
           a collocation step) non-singular, so the block has the fixed inertia (nS, nS, 0) and the
           device eliminates it by one LU of J_YX and dense products instead of a Bunch-Kaufman
           pivot chain (csrc/ato_kkt.hip, k_front_saddle; Bunch-Kaufman on the same front when
           J_YX is singular or the rows carry a delta_c).
  'chain'  the staged elimination of solver/kkt_blocks.py: front s owns interval s's variables
           and rows (a row touching two intervals joins the later one), its child is front s-1,
           the border is the root. One front per level.

This module builds the integer tables the kernels read: KKT index of every front position,
the lower-triangle entry list of every front grouped by 32-row strip with the source of
each value (Hessian entry, Jacobian entry, variable or row diagonal), the extend-add map of
every trailing position into the parent front, and the per-front storage offsets.
'''
from dataclasses import dataclass
from typing import Dict, List

import numpy as np

SRC_H, SRC_J, SRC_DX, SRC_DR = 0, 1, 2, 3
SRC_SHIFT = 29
TILE = 32
MAX_TILES = 9              # fronts up to 288 positions (kernel register tiles; nine for K = 7 leaves)


def src_code(kind: int, idx: int) -> int:
    return (kind << SRC_SHIFT) | int(idx)


@dataclass
class KKTPlan:
    n: int                      # variables
    m: int                      # rows
    dim: int                    # n + m
    ordering: str
    n_fronts: int
    n_levels: int
    level_ptr: np.ndarray       # [L+1] fronts of level l: level_ptr[l] .. level_ptr[l+1]-1
    level_tiles: np.ndarray     # [L] 32-wide tiles of the largest front of the level
    pos_ptr: np.ndarray         # [F+1] into pos_index / parent_pos
    n_own: np.ndarray           # [F]
    pos_index: np.ndarray       # [P] KKT index of every front position (own first)
    parent_pos: np.ndarray      # [P] trailing position -> position in the parent front (-1: own)
    parent: np.ndarray          # [F] parent front (-1: root)
    child_ptr: np.ndarray       # [F+1] into child_list
    child_list: np.ndarray      # [C] children of every front, ascending
    ent_ptr: np.ndarray         # [F * MAX_TILES + 1] entries of (front, strip)
    ent_pos: np.ndarray         # [E] (pa << 16) | pb with pa >= pb
    ent_src: np.ndarray         # [E, 2] source codes (-1: none)
    l_off: np.ndarray           # [F] offset of the front's factor columns (doubles, per instance)
    l_size: int                 # doubles of factor columns per instance
    piv_off: np.ndarray         # [F] offset of the front's pivot records (per instance)
    cb_off: np.ndarray          # [F] offset of the front's contribution block (tq x tq doubles)
    cb_size: int
    sc_off: np.ndarray          # [F] offset of the front's solve contribution (tq doubles)
    sc_size: int
    block_sizes: np.ndarray     # [F] own + trailing
    n_sad: np.ndarray           # [F] saddle fronts: nS (own = nS states, then their nS defect rows); else 0
    kres_ptr: np.ndarray        # [dim+1] CSR of the whole K (both triangles) for residuals r - K x
    kres_col: np.ndarray        # [nnz_K] column (KKT index), ascending within a row
    kres_src: np.ndarray        # [nnz_K] source code of the value (a diagonal with two sources: two entries)

    @property
    def max_block(self) -> int:
        return int(self.block_sizes.max())

    @property
    def tiles(self) -> int:
        return int(self.level_tiles.max())

    def front_positions(self, f: int) -> np.ndarray:
        return self.pos_index[self.pos_ptr[f]:self.pos_ptr[f + 1]]

    def children(self, f: int) -> np.ndarray:
        return self.child_list[self.child_ptr[f]:self.child_ptr[f + 1]]


def row_span(n, m, var_stage, j_row_ptr, j_col):
    ''' (lowest, highest) interval touched by every row; empty rows -> (0, 0) '''
    var_stage = np.asarray(var_stage)
    jr = np.repeat(np.arange(m), np.diff(np.asarray(j_row_ptr)))
    st = var_stage[np.asarray(j_col)]
    lo = np.full(m, np.iinfo(np.int64).max)
    hi = np.full(m, -1)
    np.minimum.at(lo, jr, st)
    np.maximum.at(hi, jr, st)
    empty = hi < 0
    lo[empty], hi[empty] = 0, 0
    return lo, hi


def row_stages(n, m, var_stage, j_row_ptr, j_col) -> np.ndarray:
    ''' stage of every row in the 'chain' ordering: the later stage of a row touching one or two
    neighbouring stages, -1 for border rows (same rule as solver/kkt_blocks.BlockKKT) '''
    lo, hi = row_span(n, m, var_stage, j_row_ptr, j_col)
    return np.where(hi - lo <= 1, hi, -1)


def _fronts_chain(n, var_stage, lo, hi):
    S = int(var_stage.max()) + 1
    rs = np.where(hi - lo <= 1, hi, -1)
    own = [np.concatenate([np.nonzero(var_stage == s)[0], n + np.nonzero(rs == s)[0]]) for s in range(S)]
    children: List[List[int]] = [[s - 1] if s > 0 else [] for s in range(S)]
    border = n + np.nonzero(rs < 0)[0]
    own.append(border)
    children.append([S - 1])
    return own, children


def collocation_saddle(N, K1, nv, nz, m, j_row_ptr, j_col):
    '''
    Saddle pairs of a collocation transcription, from the Jacobian structure alone: the states of
    nodes 1..K of every interval (variables N + (n K1 + k) nv + [0, nz)) and the rows that are
    their ODE defects. The defect of state component c at node k of interval n,
        sum_j C_jk z_j[c] - h_n f_c(z_k, u_k) = 0,
    is the row with entries on component c at EVERY node of the interval (the collocation
    derivative), on other node variables of node k only (f_c), and on nothing of another interval.
    (The s-dot rows have no f term; a gate row has no single node.) Returns (cols, rows), the
    defect of (n, k, c) paired with state (n, k, c), or None when some (n, k >= 1, c) has no unique
    defect row (RK4 steps, other transcriptions).
    '''
    j_row_ptr = np.asarray(j_row_ptr, np.int64)
    j_col = np.asarray(j_col, np.int64)
    if K1 < 2:
        return None
    jr = np.repeat(np.arange(m), np.diff(j_row_ptr))
    node_var = j_col >= N
    q = np.where(node_var, (j_col - N) // nv, -1)          # node of the entry
    comp = np.where(node_var, (j_col - N) % nv, -1)
    stage = np.where(node_var, q // K1, j_col)              # h_n -> n
    lo = np.full(m, np.iinfo(np.int64).max)
    hi = np.full(m, -1)
    np.minimum.at(lo, jr, stage)
    np.maximum.at(hi, jr, stage)
    found = {}
    for c in range(nz):
        # per row: bit k set when the row has an entry on component c (resp. another node
        # variable) of node k of its interval
        on_c = node_var & (comp == c)
        bits_c = np.zeros(m, np.int64)
        np.bitwise_or.at(bits_c, jr[on_c], np.left_shift(1, q[on_c] % K1))
        other = node_var & (comp != c)
        bits_o = np.zeros(m, np.int64)
        np.bitwise_or.at(bits_o, jr[other], np.left_shift(1, q[other] % K1))
        single = (bits_o > 0) & ((bits_o & (bits_o - 1)) == 0)
        for r in np.nonzero((bits_c == (1 << K1) - 1) & (lo == hi) & single)[0]:
            k = int(bits_o[r]).bit_length() - 1
            key = (int(lo[r]), k, c)
            if k == 0 or key in found:
                return None
            found[key] = int(r)
    cols, rows = [], []
    for st in range(N):
        for k in range(1, K1):
            for c in range(nz):
                if (st, k, c) not in found:
                    return None
                cols.append(N + (st * K1 + k) * nv + c)
                rows.append(found[(st, k, c)])
    return np.asarray(cols, np.int64), np.asarray(rows, np.int64)


HUB_MIN_ROWS = 3           # border rows of a hub reach this many distinct intervals (eliminated at the root)


def cpc_node_groups(spec):
    ''' the CPC progress variables (lambda, mu, nu per waypoint) of every collocation node, for the node
    chain of build_plan (raceline/problem.py _cpc_block: laid out node by node after all node variables);
    None without CPC '''
    if getattr(spec, 'cpc', None) is None:
        return None
    w = 3 * spec.cpc_m
    return [spec.cpc_off + q * w + np.arange(w) for q in range(spec.P)]


def _fronts_nd(n, var_stage, lo, hi, j_row_ptr, j_col, split_pairs=True, saddle=None, node_groups=None):
    S = int(var_stage.max()) + 1
    m = len(lo)
    jr = np.repeat(np.arange(m), np.diff(np.asarray(j_row_ptr)))
    jc = np.asarray(j_col)
    # hubs: variables on many rows that span more than two intervals -- the first step size h_n0 of a
    # global raceline's gate phase, which the equal-step rows h_n2 - h_n0 = 0 tie to every step of the
    # phase (base_raceline.py:897-905). As border rows those would all sit in the root front (514
    # positions for race.py's 490 RK4 steps, over the device's 256). Instead a hub is eliminated at the
    # root like the root anchors below, and the rows' spans are taken without it: h_n2 - h_n0 becomes
    # an interior row of interval n2, whose leaf hands h_n0 up as one trailing position.
    # (a hub's border rows reach at least HUB_MIN_ROWS distinct far intervals; a closed line's closure
    # rows all reach interval 0 and stay with the root anchors)
    bsel = (hi - lo > 1)[jr]
    bv, br = jc[bsel], jr[bsel]
    far = np.where(var_stage[bv] == lo[br], hi[br], lo[br])
    pairs = np.unique(np.stack([bv, far]), axis=1)
    hub = np.bincount(pairs[0], minlength=n) >= HUB_MIN_ROWS
    if hub.any():
        kept = ~hub[jc]
        st = var_stage[jc]
        lo2 = np.full(m, np.iinfo(np.int64).max)
        hi2 = np.full(m, -1)
        np.minimum.at(lo2, jr[kept], st[kept])
        np.maximum.at(hi2, jr[kept], st[kept])
        some = hi2 >= 0                          # rows with a non-hub entry take the reduced span
        lo, hi = np.where(some, lo2, lo), np.where(some, hi2, hi)
    link = hi - lo == 1
    interior = hi == lo
    # anchors of boundary j: the variables of interval j touched by its link rows
    anchor = np.zeros(n, bool)
    sel = link[jr] & (var_stage[jc] == hi[jr])
    anchor[jc[sel]] = True
    anchor &= ~hub
    # root anchors: the interval-0 variables that border rows touch (a closed line's closure rows
    # tie node 0 to the last node). They are eliminated in the border front, so the closure rows
    # no longer couple to leaf 0 -- its block shrinks from 182 to 166 positions on the racetrack,
    # the size class of the other leaves -- and they reach the root as trailing positions of the
    # leaf and of the separators on its path.
    border_row = hi - lo > 1
    root_anchor = np.zeros(n, bool)
    rsel = border_row[jr] & (var_stage[jc] == 0)
    root_anchor[jc[rsel]] = True
    root_anchor &= ~anchor
    root_anchor |= hub
    # interior rows whose every entry sits on anchors (e.g. a global-frame gate row on Z[n,0][:3],
    # whose position the continuity rows make anchors) have no variable inside the leaf: in the
    # leaf their own column would hold only the row diagonal (a zero pivot for an equality row,
    # i.e. a spurious singular KKT). They join the separator that owns their anchors instead.
    has_inner = np.zeros(m, bool)
    has_inner[jr[interior[jr] & ~anchor[jc] & ~root_anchor[jc]]] = True
    anchor_only = interior & ~has_inner & (lo >= 1)
    root_only = interior & ~has_inner & (lo == 0) & root_anchor.any()    # rows on root anchors only
    own: List[np.ndarray] = []
    children: List[List[int]] = []
    # isolated pairs: an interior variable whose only Jacobian entry is in an interior row of its
    # interval (the input rates dU_k and their defect rows dU_k - sum_j C_jk U_j / h: the row is the
    # variable's only coupling besides its Hessian diagonal and h). The pairs of an interval form a
    # child front of the leaf: eliminated first, they leave a smaller leaf block (fewer register
    # tiles, cheaper pivot steps) and a short chain of small-front steps instead
    pre = [np.zeros(0, np.int64) for _ in range(S)]
    # node groups (CPC progress variables of every node, cpc_node_groups): node of every grouped variable
    gnode = np.full(n, -1, np.int64)
    if node_groups is not None:
        for q, g in enumerate(node_groups):
            gnode[np.asarray(g, np.int64)] = q
    npairs: Dict[int, List[tuple]] = {}             # pairs of a grouped variable: pre-front of its node front
    if split_pairs:
        cnt = np.bincount(jc, minlength=n)
        used = np.zeros(m, bool)
        pairs: List[List[int]] = [[] for _ in range(S)]
        for e in np.nonzero(cnt[jc] == 1)[0]:
            v, r = int(jc[e]), int(jr[e])
            st = int(var_stage[v])
            if anchor[v] or root_anchor[v] or used[r] or root_only[r] or not (interior[r] and lo[r] == st):
                continue
            used[r] = True
            if gnode[v] >= 0:
                npairs.setdefault(int(gnode[v]), []).append((v, r))
            else:
                pairs[st].append((v, r))
        for st in range(S):
            if pairs[st]:
                pre[st] = np.concatenate([np.sort([v for v, _ in pairs[st]]), n + np.sort([r for _, r in pairs[st]])])
    pre_id = [-1] * S
    for st in range(S):                          # pre-fronts first (children precede parents)
        if len(pre[st]):
            pre_id[st] = len(own)
            own.append(pre[st])
            children.append([])
    # node chain (CPC, config 5): the progress variables of node q and the rows that touch progress
    # variables only (order rows, progress rows lambda_{q+1} - lambda_q + mu_q = 0: they couple node q to
    # q + 1 only) form a front of node q; inside an interval the node fronts are a chain, each the child
    # of the next and the last the child of the leaf, with the node's (nu, complementarity row) pairs as a
    # pre-front below it. In the leaf they would add ~200 positions (fig-8 56 x 4 with eight waypoints:
    # 360, over the kernels' 288); as a chain each front holds ~31 own positions and trails the node
    # positions of its interval and the next node's lambda.
    chain_last: List[List[int]] = [[] for _ in range(S)]
    in_chain = np.zeros(n + m, bool)
    if node_groups is not None:
        gvar = gnode >= 0
        rmin = np.full(m, np.iinfo(np.int64).max)
        np.minimum.at(rmin, jr, np.where(gvar[jc], gnode[jc], np.iinfo(np.int64).max))
        n_non = np.bincount(jr[~gvar[jc]], minlength=m)           # entries on other variables
        paired = np.zeros(m, bool)
        for lst in npairs.values():
            paired[[r for _, r in lst]] = True
        crow = interior & ~anchor_only & ~root_only & (n_non == 0) & (rmin < len(node_groups)) & ~paired
        rows_of: Dict[int, List[int]] = {}
        for r in np.nonzero(crow)[0]:
            rows_of.setdefault(int(rmin[r]), []).append(int(r))
        pending: Dict[int, List[int]] = {}         # fronts of an interval waiting for the next chain front
        for q, g in enumerate(node_groups):
            g = np.asarray(g, np.int64)
            st = int(var_stage[g[0]])
            pv = {v for v, _ in npairs.get(q, [])}
            vs = np.array([v for v in g if not anchor[v] and not root_anchor[v] and v not in pv], np.int64)
            rs = np.array(sorted(r for r in rows_of.get(q, []) if lo[r] == st), np.int64)
            kids = pending.pop(st, [])
            if q in npairs:
                pl = npairs[q]
                kids.append(len(own))
                own.append(np.concatenate([np.sort([v for v, _ in pl]), n + np.sort([r for _, r in pl])]))
                children.append([])
                for v, r in pl:
                    in_chain[v] = True
                    in_chain[n + r] = True
            if len(vs) or len(rs):
                pending[st] = [len(own)]
                own.append(np.concatenate([vs, n + rs]))
                children.append(kids)
                in_chain[vs] = True
                in_chain[n + rs] = True
            else:
                pending[st] = kids
        for st, fl in pending.items():
            chain_last[st] = fl
    # saddle fronts: the states of nodes 1..K and their ODE defect rows (collocation_saddle), when
    # every one of them lies inside the leaf (not an anchor, not in a pre-front pair)
    sad_id = [-1] * S
    n_sad: List[int] = [0] * len(own)
    sad = [np.zeros(0, np.int64) for _ in range(S)]
    if saddle is not None:
        scols, srows = (np.asarray(a, np.int64) for a in saddle)
        for st in range(S):
            xs = np.sort(scols[var_stage[scols] == st])
            ys = np.sort(srows[(lo[srows] == st) & (hi[srows] == st)])
            if not len(xs) or len(xs) != len(ys) or len(xs) > 64:
                continue
            inner_ok = not (anchor[xs].any() or root_anchor[xs].any() or (~interior[ys]).any() or
                            anchor_only[ys].any() or root_only[ys].any())
            if len(pre[st]):
                inner_ok = inner_ok and not np.isin(np.concatenate([xs, n + ys]), pre[st]).any()
            if not inner_ok:
                continue
            sad[st] = np.concatenate([xs, n + ys])
            sad_id[st] = len(own)
            own.append(sad[st])
            children.append([])
            n_sad.append(len(xs))
    leaf_id = []
    for st in range(S):                          # leaves
        inner = np.concatenate([np.nonzero((var_stage == st) & ~anchor & ~root_anchor)[0],
                                n + np.nonzero(interior & ~anchor_only & ~root_only & (lo == st))[0]])
        if len(pre[st]):
            inner = inner[~np.isin(inner, pre[st])]
        if len(sad[st]):
            inner = inner[~np.isin(inner, sad[st])]
        inner = inner[~in_chain[inner]]
        leaf_id.append(len(own))
        own.append(inner)
        children.append([c for c in (pre_id[st], sad_id[st]) if c >= 0] + chain_last[st])

    def sep(j):
        return np.concatenate([np.nonzero((var_stage == j) & anchor)[0],
                               n + np.nonzero((link | anchor_only) & (hi == j))[0]])

    def build(a, b):                            # subtree over intervals a..b (boundaries a+1..b)
        if a == b:
            return leaf_id[a]
        j = (a + b + 1) // 2
        left, right = build(a, j - 1), build(j, b)
        own.append(sep(j))
        children.append([left, right])
        return len(own) - 1

    top = build(0, S - 1)
    border = np.concatenate([np.nonzero(root_anchor)[0], n + np.nonzero(border_row | root_only)[0]])
    if len(border):
        own.append(border)
        children.append([top])
    n_sad += [0] * (len(own) - len(n_sad))
    return own, children, n_sad


def build_plan(n: int, m: int, var_stage, j_row_ptr, j_col, h_row_ptr, h_col, ordering: str = 'nd',
               split_pairs: bool = True, saddle=None, node_groups=None) -> KKTPlan:
    '''
    saddle: optional (cols, rows) saddle pairs (collocation_saddle) for the 'nd' ordering: every
    interval's set becomes a saddle front, a child of the interval's leaf.
    node_groups: optional per-node variable groups (cpc_node_groups) eliminated as a chain of node
    fronts below every leaf ('nd' ordering).
    '''
    var_stage = np.asarray(var_stage, np.int64)
    j_row_ptr = np.asarray(j_row_ptr, np.int64)
    j_col = np.asarray(j_col, np.int64)
    h_row_ptr = np.asarray(h_row_ptr, np.int64)
    h_col = np.asarray(h_col, np.int64)
    jr = np.repeat(np.arange(m), np.diff(j_row_ptr))
    hr = np.repeat(np.arange(n), np.diff(h_row_ptr))
    if len(hr) and np.any(var_stage[hr] != var_stage[h_col]):
        raise ValueError('Hessian couples different stages; the staged KKT does not apply')
    lo, hi = row_span(n, m, var_stage, j_row_ptr, j_col)
    if ordering == 'nd':
        own, children, n_sad = _fronts_nd(n, var_stage, lo, hi, j_row_ptr, j_col, split_pairs, saddle, node_groups)
    elif ordering == 'chain':
        own, children = _fronts_chain(n, var_stage, lo, hi)
        n_sad = [0] * len(own)
    else:
        raise ValueError(f'unknown KKT ordering {ordering!r}')
    F0 = len(own)
    cover = np.concatenate(own)
    if not np.array_equal(np.sort(cover), np.arange(n + m)):
        raise AssertionError('KKT fronts do not partition the KKT indices')

    # ---- levels (children first), fronts renumbered level by level
    level = np.zeros(F0, np.int64)
    for f in range(F0):                         # children always precede parents in creation order
        if children[f]:
            level[f] = 1 + max(level[c] for c in children[f])
    order = np.lexsort((np.arange(F0), level))
    new_id = np.empty(F0, np.int64)
    new_id[order] = np.arange(F0)
    own = [own[f] for f in order]
    children = [sorted(int(new_id[c]) for c in children[f]) for f in order]
    n_sad = np.asarray([n_sad[f] for f in order], np.int64)
    level = level[order]
    F = F0
    parent = np.full(F, -1, np.int64)
    for f in range(F):
        for c in children[f]:
            parent[c] = f

    # ---- adjacency of the KKT graph (structural nonzeros, both triangles)
    dim = n + m
    adj_r = np.concatenate([hr, h_col, jr + n, j_col])
    adj_c = np.concatenate([h_col, hr, j_col, jr + n])
    keep = adj_r != adj_c
    adj_r, adj_c = adj_r[keep], adj_c[keep]
    srt = np.argsort(adj_r, kind='stable')
    adj_r, adj_c = adj_r[srt], adj_c[srt]
    adj_ptr = np.searchsorted(adj_r, np.arange(dim + 1))

    # ---- trailing sets by symbolic elimination in front order
    owner = np.empty(dim, np.int64)
    for f in range(F):
        owner[own[f]] = f
    trailing: List[np.ndarray] = []
    eliminated = np.zeros(dim, bool)
    for f in range(F):
        o = own[f]
        isown = np.zeros(dim, bool)
        isown[o] = True
        # neighbours eliminated earlier were assembled into a descendant and reach this front
        # through the contribution blocks; the children's trailing positions must all be live
        nb = np.concatenate([adj_c[adj_ptr[i]:adj_ptr[i + 1]] for i in o] + [np.zeros(0, np.int64)])
        nb = nb[~eliminated[nb]]
        ct = np.concatenate([trailing[c] for c in children[f]] + [np.zeros(0, np.int64)])
        if eliminated[ct].any():
            raise AssertionError(f'front {f}: a child hands over positions eliminated outside its ancestry')
        cand = np.unique(np.concatenate([nb, ct]))
        cand = cand[~isown[cand]]
        if n_sad[f] > 0:
            # saddle front: trailing positions coupled to the states only, then to states and defect
            # rows, then to the defect rows only, so that K_TX and K_TY are row ranges [0, tx) and
            # [T - ty, T) (k_front_saddle keeps only those rows)
            ns = int(n_sad[f])
            cls = np.zeros(len(cand), np.int64)
            for q, i in enumerate(cand):
                nbi = adj_c[adj_ptr[i]:adj_ptr[i + 1]]
                to_x = np.isin(nbi, o[:ns]).any()
                to_y = np.isin(nbi, o[ns:]).any()
                cls[q] = 0 if not to_y else (1 if to_x else 2)
            cand = cand[np.lexsort((cand, cls))]
        trailing.append(cand)
        eliminated[o] = True
    if any(len(trailing[f]) for f in range(len(own)) if parent[f] < 0):
        raise AssertionError('a root front has trailing positions')
    # every trailing position must be eliminated by an ancestor, and sit in the parent's front
    pos_of: List[Dict[int, int]] = []
    for f in range(F):
        pos_of.append({int(i): q for q, i in enumerate(np.concatenate([own[f], trailing[f]]))})
    for f in range(F):
        if len(trailing[f]):
            p = int(parent[f])
            if p < 0 or any(int(i) not in pos_of[p] for i in trailing[f]):
                raise AssertionError(f'front {f}: trailing positions outside the parent front')

    sizes = np.array([len(own[f]) + len(trailing[f]) for f in range(F)])
    if sizes.max(initial=0) > MAX_TILES * TILE:
        raise ValueError(f'KKT front of {sizes.max()} positions exceeds the device limit {MAX_TILES * TILE}')
    n_levels = int(level.max()) + 1
    level_ptr = np.searchsorted(level, np.arange(n_levels + 1))
    level_tiles = np.array([max(1, -(-int(sizes[level_ptr[l]:level_ptr[l + 1]].max()) // TILE))
                            for l in range(n_levels)])

    # ---- entries: each original entry (i, j) belongs to the front eliminating the earlier of i, j
    rank = np.empty(dim, np.int64)               # elimination rank (front order, then own order)
    r0 = 0
    for f in range(F):
        rank[own[f]] = r0 + np.arange(len(own[f]))
        r0 += len(own[f])
    ent: List[Dict] = [dict() for _ in range(F)]

    def add(i, j, code):
        f = int(owner[i] if rank[i] <= rank[j] else owner[j])
        pa, pb = pos_of[f][int(i)], pos_of[f][int(j)]
        if pa < pb:
            pa, pb = pb, pa
        ent[f].setdefault((pa, pb), []).append(code)

    for e in range(len(h_col)):                 # Hessian (lower)
        add(int(hr[e]), int(h_col[e]), src_code(SRC_H, e))
    for j in range(n):                          # variable diagonal
        add(j, j, src_code(SRC_DX, j))
    for e in range(len(j_col)):                 # Jacobian (row i, variable j)
        add(n + int(jr[e]), int(j_col[e]), src_code(SRC_J, e))
    for i in range(m):                          # row diagonal
        add(n + i, n + i, src_code(SRC_DR, i))

    ent_ptr = [0]
    ent_pos, ent_src = [], []
    for f in range(F):
        strips = [[] for _ in range(MAX_TILES)]
        for k in sorted(ent[f].keys(), key=lambda k: (k[0] // TILE, k[0], k[1])):
            srcs = ent[f][k]
            if len(srcs) > 2:
                raise ValueError(f'KKT entry {k} of front {f} has {len(srcs)} sources')
            strips[k[0] // TILE].append((k, srcs))
        for I in range(MAX_TILES):
            for (pa, pb), srcs in strips[I]:
                ent_pos.append((pa << 16) | pb)
                ent_src.append([srcs[0], srcs[1] if len(srcs) > 1 else -1])
            ent_ptr.append(len(ent_pos))

    # ---- positions, extend-add map, children
    pos_index = np.concatenate([np.concatenate([own[f], trailing[f]]) for f in range(F)])
    pos_ptr = np.concatenate([[0], np.cumsum(sizes)])
    parent_pos = np.full(len(pos_index), -1, np.int64)
    for f in range(F):
        p = int(parent[f])
        for q, i in enumerate(trailing[f]):
            parent_pos[pos_ptr[f] + len(own[f]) + q] = pos_of[p][int(i)]
    child_ptr = np.concatenate([[0], np.cumsum([len(c) for c in children])])
    child_list = np.asarray([c for cs in children for c in cs], np.int64)

    # ---- CSR of K for the residual kernel (refinement): every structural entry in both triangles
    rr, cc, ss = [], [], []
    for e in range(len(h_col)):
        r_, c_ = int(hr[e]), int(h_col[e])
        rr.append(r_), cc.append(c_), ss.append(src_code(SRC_H, e))
        if r_ != c_:
            rr.append(c_), cc.append(r_), ss.append(src_code(SRC_H, e))
    for j in range(n):
        rr.append(j), cc.append(j), ss.append(src_code(SRC_DX, j))
    for e in range(len(j_col)):
        i, j = n + int(jr[e]), int(j_col[e])
        rr.append(i), cc.append(j), ss.append(src_code(SRC_J, e))
        rr.append(j), cc.append(i), ss.append(src_code(SRC_J, e))
    for i in range(m):
        rr.append(n + i), cc.append(n + i), ss.append(src_code(SRC_DR, i))
    rr, cc, ss = np.asarray(rr), np.asarray(cc), np.asarray(ss)
    o = np.lexsort((ss, cc, rr))
    kres_ptr = np.searchsorted(rr[o], np.arange(dim + 1))

    # ---- per-instance storage: compact factor columns, pivot records, contribution blocks
    n_own = np.array([len(o) for o in own])
    tq = sizes - n_own
    l_sz = n_own * sizes - n_own * (n_own + 1) // 2
    # a saddle front stores either the Bunch-Kaufman columns (fallback) or K_SS^-1 (2nS x 2nS) and
    # W = K_TS K_SS^-1 (tq x 2nS)
    l_sz = np.maximum(l_sz, np.where(n_sad > 0, (2 * n_sad) ** 2 + tq * 2 * n_sad, 0))
    l_off = np.concatenate([[0], np.cumsum(l_sz)])
    piv_off = np.concatenate([[0], np.cumsum(n_own)])
    cb_off = np.concatenate([[0], np.cumsum(tq * tq)])
    sc_off = np.concatenate([[0], np.cumsum(tq)])
    i32 = lambda a: np.asarray(a, np.int32)  # noqa: E731
    return KKTPlan(n=n, m=m, dim=dim, ordering=ordering, n_fronts=F, n_levels=n_levels,
                   level_ptr=i32(level_ptr), level_tiles=i32(level_tiles), pos_ptr=i32(pos_ptr), n_own=i32(n_own),
                   pos_index=i32(pos_index), parent_pos=i32(parent_pos), parent=i32(parent),
                   child_ptr=i32(child_ptr), child_list=i32(child_list),
                   ent_ptr=i32(ent_ptr), ent_pos=i32(ent_pos), ent_src=i32(ent_src).reshape(-1, 2),
                   l_off=np.asarray(l_off[:-1], np.int64), l_size=int(l_off[-1]),
                   piv_off=i32(piv_off[:-1]), cb_off=np.asarray(cb_off[:-1], np.int64), cb_size=int(cb_off[-1]),
                   sc_off=i32(sc_off[:-1]), sc_size=int(sc_off[-1]), block_sizes=i32(sizes), n_sad=i32(n_sad),
                   kres_ptr=i32(kres_ptr), kres_col=i32(cc[o]), kres_src=i32(ss[o]))
