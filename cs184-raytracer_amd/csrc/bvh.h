// Per-mesh linear BVH (Morton-ordered, Karras-style binary radix splits), built on the
// host once at rt_scene_create and flattened for upload.  New design: the reference
// scans every face of a mesh (geometry.cpp:78-124).  Traversal must reproduce that
// scan's closest-hit choice exactly (see trace kernels), so boxes are padded outward.
#pragma once
#include <vector>
#include "device_types.h"
#include "scene_host.h"

namespace rtamd {

struct FlatScene {
	std::vector<DGeom> geoms;
	std::vector<DMaterial> materials;
	std::vector<DLight> lights;
	std::vector<DFaceGeo> face_geo;
	std::vector<DFaceNrm> face_nrm;
	std::vector<DBvhNode> nodes;
	// geometry indices in shadow-test order: the occlusion query is an `any` over the
	// geometries, so cheap ones (spheres, linearly scanned meshes) go first
	std::vector<int32_t> shadow_order;
	int32_t n_may_raise = 0;
	DCamera camera;
	int max_bvh_depth = 0;
};

// Flattens the host scene, building an LBVH for every mesh with > kLinearFaces faces.
FlatScene flatten_scene(const Scene& s);

}  // namespace rtamd
