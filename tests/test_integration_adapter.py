"""The reference-side binding (include/integration/GpuIterativeClosestPointOptimizer.h) against the reference's own
headers: it cannot be compiled here (the reference needs the system Eigen3 this image lacks), so every reference
identifier it names -- namespaces, types, struct fields, methods -- is checked to exist where it claims, and its
optimize / optimize_loop / get_last_stats signatures to equal the reference's (IterativeClosestPointOptimizer.h:42-43,
:159-227; AdaptiveMEstimator.h:27-41).  Skipped when /root/reference is absent (the GPU box).
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src"
ADAPTER = os.path.join(ROOT, "include", "integration", "GpuIterativeClosestPointOptimizer.h")

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")


def _read(rel):
    with open(os.path.join(REF, rel)) as f:
        return f.read()


def _strip_comments(s):
    s = re.sub(r"/\*.*?\*/", "", s, flags=re.S)
    return re.sub(r"//[^\n]*", "", s)


def _body(src, head_re):
    """Text of the brace block that follows the first match of head_re."""
    m = re.search(head_re, src)
    assert m, head_re
    i = src.index("{", m.end() - 1)
    depth = 0
    for j in range(i, len(src)):
        depth += {"{": 1, "}": -1}.get(src[j], 0)
        if depth == 0:
            return src[i:j + 1]
    raise AssertionError("unbalanced " + head_re)


def _norm(sig):
    return re.sub(r"\s+", " ", sig).replace("( ", "(").replace(" )", ")").strip()


@pytest.fixture(scope="module")
def adapter():
    with open(ADAPTER) as f:
        return _strip_comments(f.read())


@pytest.fixture(scope="module")
def ref():
    return {k: _strip_comments(_read(k)) for k in (
        "optimization/IterativeClosestPointOptimizer.h", "optimization/AdaptiveMEstimator.h",
        "database/VoxelMap.h", "database/LidarFrame.h", "util/MathUtils.h", "util/PointCloudUtils.h")}


def test_includes_exist(adapter):
    for inc in re.findall(r'#include "([^"]+)"', adapter):
        if inc == "lo_icp.h":
            assert os.path.exists(os.path.join(ROOT, "include", inc))
        else:
            assert os.path.exists(os.path.join(REF, inc)), inc


def test_namespace_matches_reference(adapter, ref):
    icp = ref["optimization/IterativeClosestPointOptimizer.h"]
    # the reference declares the optimizer inside namespace lidar_slam { namespace optimization { ... } }
    assert re.search(r"namespace lidar_slam\s*\{\s*namespace optimization\s*\{", icp)
    assert re.search(r"namespace lidar_slam\s*\{\s*namespace optimization\s*\{", adapter)
    assert "lidar_odometry::" not in adapter


def test_types_exist(adapter, ref):
    icp, pko = ref["optimization/IterativeClosestPointOptimizer.h"], ref["optimization/AdaptiveMEstimator.h"]
    assert re.search(r"struct ICPConfig\s*\{", icp)
    assert re.search(r"struct AdaptiveMEstimatorConfig\s*\{", pko)
    assert re.search(r"class AdaptiveMEstimator\s*\{", pko)
    assert re.search(r"struct OptimizationStats\s*\{", _body(icp, r"class IterativeClosestPointOptimizer\s*\{"))
    assert re.search(r"class VoxelMap\s*\{", ref["database/VoxelMap.h"])
    assert re.search(r"class LidarFrame\s*\{", ref["database/LidarFrame.h"])
    assert re.search(r"using SE3f\s*=", ref["util/MathUtils.h"])
    for alias in ("PointCloudPtr", "PointCloudConstPtr"):
        assert re.search(r"using %s\s*=" % alias, ref["util/PointCloudUtils.h"] + icp), alias
    for t in ("ICPConfig", "AdaptiveMEstimatorConfig", "AdaptiveMEstimator", "IterativeClosestPointOptimizer::OptimizationStats",
              "map::VoxelMap", "database::LidarFrame", "SE3f", "util::PointCloudConstPtr", "util::PointCloudPtr"):
        assert t in adapter, t


def _members(adapter, obj_re):
    return sorted(set(re.findall(obj_re + r"(?:\.|->)\s*(\w+)", adapter)))


def test_struct_fields_exist(adapter, ref):
    icp, pko = ref["optimization/IterativeClosestPointOptimizer.h"], ref["optimization/AdaptiveMEstimator.h"]
    checks = [
        (r"\bm_config", _body(icp, r"struct ICPConfig\s*\{")),
        (r"\bcfg", _body(icp, r"struct ICPConfig\s*\{")),          # make_config's ICPConfig argument
        (r"\bp", _body(pko, r"struct AdaptiveMEstimatorConfig\s*\{")),
        (r"\bm_last_stats", _body(icp, r"struct OptimizationStats\s*\{")),
    ]
    seen = 0
    for obj, body in checks:
        names = _members(adapter, obj)
        assert names, obj
        for f in names:
            assert re.search(r"\b%s\b" % f, body), f"{obj}.{f} is not a field of the reference type"
            seen += 1
    # every field the reference's OptimizationStats has is written by the adapter
    stats = _body(icp, r"struct OptimizationStats\s*\{")
    for f in re.findall(r"(\w+)\s*=\s*[^;]+;", stats):
        assert f in _members(adapter, r"\bm_last_stats"), f
    assert seen >= 20


def test_methods_exist(adapter, ref):
    vm = _body(ref["database/VoxelMap.h"], r"class VoxelMap\s*\{")
    lf = _body(ref["database/LidarFrame.h"], r"class LidarFrame\s*\{")
    se3 = _body(ref["util/MathUtils.h"], r"class SE3\s*\{")
    pc = _body(ref["util/PointCloudUtils.h"], r"class PointCloud\s*\{")
    est = _body(ref["optimization/AdaptiveMEstimator.h"], r"class AdaptiveMEstimator\s*\{")
    checks = [
        (r"\bvm", vm), (r"\b(?:curr_frame|frame|curr_keyframe|matched_keyframe)", lf), (r"\bT", se3),
        (r"\b(?:cloud|cur|mat|feature|processed)", pc), (r"\bm_adaptive_estimator", est),
    ]
    for obj, body in checks:
        names = _members(adapter, obj)
        assert names, obj
        for m in names:
            assert re.search(r"\b%s\b" % m, body), f"{obj} -> {m} is not a member of the reference class"


def test_signatures_match_reference(adapter, ref):
    icp = ref["optimization/IterativeClosestPointOptimizer.h"]
    cls = _body(icp, r"class IterativeClosestPointOptimizer\s*\{")
    for name in ("optimize", "optimize_loop"):
        m = re.search(r"bool\s+%s\s*\(([^)]*)\)\s*;" % name, cls)
        assert m, name
        ref_types = [_norm(re.sub(r"\w+\s*$", "", a.strip())) for a in m.group(1).split(",")]
        a = re.search(r"bool\s+%s\s*\(([^)]*)\)\s*\{" % name, adapter)
        assert a, name
        ad_types = [_norm(re.sub(r"\w+\s*$", "", x.strip())) for x in a.group(1).split(",")]
        assert ad_types == ref_types, (name, ad_types, ref_types)
    assert re.search(r"const OptimizationStats& get_last_stats\(\) const", cls)
    assert re.search(r"const OptimizationStats& get_last_stats\(\) const", adapter)
    m = re.search(r"IterativeClosestPointOptimizer\(const ICPConfig& config,\s*std::shared_ptr<optimization::AdaptiveMEstimator> adaptive_estimator\)", cls)
    assert m
    assert re.search(r"GpuIterativeClosestPointOptimizer\(const ICPConfig& config, std::shared_ptr<AdaptiveMEstimator> adaptive_estimator", adapter)


def test_kernel_names_map_as_reference():
    """pko_kernel_type dispatch (AdaptiveMEstimator.cpp:128-156): every name the reference tests maps to its own
    kernel id, anything else to Cauchy -- through the library's lo_pko_kernel_from_name (no GPU call)."""
    from lidar_odometry_amd import lib
    src = _read("optimization/AdaptiveMEstimator.cpp")
    body = _body(src, r"double AdaptiveMEstimator::pko_kernel_weight\(")
    names = re.findall(r'kernel_type == "(\w+)"', body)
    assert names == ["huber", "cauchy", "tukey", "welsch", "gemanMcClure", "pseudoHuber"]
    L = lib()
    got = [L.lo_pko_kernel_from_name(n.encode()) for n in names]
    assert got == list(range(6))
    assert L.lo_pko_kernel_from_name(b"Huber") == 1 and L.lo_pko_kernel_from_name(b"") == 1
    assert L.lo_pko_kernel_from_name(None) == 1


def test_mutable_accessors_exist_for_unprojected_output(ref):
    """from_row_major writes the device pose through SE3's non-const Rotation() / Translation() and SO3's non-const
    Matrix() (no SO3(Matrix3f) projection on the output path, tests/test_adapter_pose.py): those accessors exist."""
    mu = ref["util/MathUtils.h"]
    assert re.search(r"\bSO3&\s+Rotation\(\)\s*\{", mu)
    assert re.search(r"Eigen::Vector3f&\s+Translation\(\)\s*\{", mu)
    assert re.search(r"Eigen::Matrix3f&\s+Matrix\(\)\s*\{", mu)
