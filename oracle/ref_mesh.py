'''
ORACLE (test infrastructure only): point-to-triangle-mesh signed distance in numpy, restating
what MeshObstacle gets from trimesh (drone3d/obstacles/mesh_obstacle.py:38-41: -signed_distance,
positive outside). Independent of the product kernel's algorithm: distance = min over triangles
of (in-plane projection if it falls inside the triangle, else the nearest of the three edge
segments); inside = odd number of crossings of a ray along a DIFFERENT direction than the kernel.
trimesh itself is not installed here; parity is against this restatement.
'''
import numpy as np


def _seg_dist2(p, a, b):
    ab = b - a
    t = np.clip(np.einsum('ij,ij->i', p - a, ab) / np.maximum(np.einsum('ij,ij->i', ab, ab), 1e-300), 0, 1)
    d = p - (a + t[:, None] * ab)
    return np.einsum('ij,ij->i', d, d)


def point_mesh_distance(p, V, F):
    ''' unsigned distance of one point p (3,) to the mesh (V, F) '''
    a, b, c = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    n = np.cross(b - a, c - a)
    nn = np.einsum('ij,ij->i', n, n)
    P = np.broadcast_to(p, a.shape)
    t = np.einsum('ij,ij->i', P - a, n) / np.maximum(nn, 1e-300)
    q = P - t[:, None] * n                                          # projection onto the plane
    # barycentric inside test
    c0 = np.einsum('ij,ij->i', np.cross(b - a, q - a), n)
    c1 = np.einsum('ij,ij->i', np.cross(c - b, q - b), n)
    c2 = np.einsum('ij,ij->i', np.cross(a - c, q - c), n)
    inside = (c0 >= 0) & (c1 >= 0) & (c2 >= 0)
    d_plane = t * t * nn
    d_edge = np.minimum(np.minimum(_seg_dist2(P, a, b), _seg_dist2(P, b, c)), _seg_dist2(P, c, a))
    return np.sqrt(np.where(inside, np.minimum(d_plane, d_edge), d_edge).min())


def point_inside(p, V, F, direction=(0.2672612419124244, -0.5345224838248488, 0.8017837257372732)):
    ''' ray-crossing parity along `direction` '''
    d = np.asarray(direction, float)
    a, b, c = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    e1, e2 = b - a, c - a
    pv = np.cross(np.broadcast_to(d, e2.shape), e2)
    det = np.einsum('ij,ij->i', e1, pv)
    ok = np.abs(det) > 1e-300
    inv = np.where(ok, 1.0 / np.where(ok, det, 1.0), 0.0)
    tv = p - a
    u = np.einsum('ij,ij->i', tv, pv) * inv
    qv = np.cross(tv, e1)
    v = (qv @ d) * inv
    t = np.einsum('ij,ij->i', e2, qv) * inv
    hit = ok & (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t > 0)
    return bool(hit.sum() % 2)


def signed_distance(X, V, F):
    ''' positive outside, negative inside (MeshObstacle.signed_distance) '''
    X = np.atleast_2d(X)
    return np.array([-point_mesh_distance(x, V, F) if point_inside(x, V, F) else point_mesh_distance(x, V, F)
                     for x in X])
