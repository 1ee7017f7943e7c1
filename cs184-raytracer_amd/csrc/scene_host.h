// Host-side scene model and .rti/.obj ingest (C++).
//
// The reference builds a polymorphic Scene (scene.h:9-39) from RTIParser / OBJParser
// (parsers.cpp:93-374).  Here the same grammar produces flat, device-ready arrays:
// per-geometry affine transforms (forward, inverse, det sign), one material per
// geometry, pre-transformed lights and camera corners, and all mesh faces in object
// space.  Every transform is evaluated in the reference's Eigen 3.2.2 operation order
// (see xform.h) so the uploaded bits equal the reference's.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace rtamd {

enum GeomKind : int32_t { GEOM_SPHERE = 0, GEOM_MESH = 1 };
enum LightKind : int32_t { LIGHT_POINT = 0, LIGHT_DIRECTIONAL = 1, LIGHT_AMBIENT = 2 };

struct Material {  // rtbase.h:30-39
	double ka[3] = {0, 0, 0}, kd[3] = {0, 0, 0}, ks[3] = {0, 0, 0}, kr[3] = {0, 0, 0};
	double ns = 0;
	double kt[3] = {0, 0, 0};
	double ior = 0;
};

struct Affine {  // Transform<double,3,Affine>: rows 0..2 of the 4x4 (last row 0 0 0 1)
	double m[3][4];
};

struct Geometry {
	GeomKind kind;
	Affine fwd, inv;
	double det;            // forwardTransform().matrix().determinant() (rtbase.h:58-60)
	Material mat;
	double center[4];      // sphere (geometry.h:21)
	float radius;          // sphere, float as in geometry.h:22
	int64_t face_begin = 0, face_count = 0;  // mesh faces in Scene::faces
	bool box_valid = false;  // Mesh::updateBoundingBox ran (obj meshes only, parsers.cpp:119)
	double bb_min[4] = {0, 0, 0, 0}, bb_max[4] = {0, 0, 0, 0};
};

struct Face {  // Mesh::Face (geometry.h:32): object-space points + normals
	double p[3][4];
	double n[3][4];
};

struct Light {  // lights.h
	LightKind kind;
	double color[3];
	double vec[4];      // point: fwd*point (w=1); directional: fwd*direction (w=0)
	double falloff = 0;
	Affine fwd;         // the light's forwardTransform (lights.h:31,59)
	double raw[4];      // PointLight::point_ / DirectionalLight::direction_ before fwd
};

struct Scene {
	bool has_camera = false;
	double cam[5][4];   // fwd*{eye, lowerLeft, lowerRight, upperLeft, upperRight} (rtbase.h:86-95)
	double cam_raw[5][4];  // the same points before the camera's forwardTransform
	Affine cam_fwd;
	std::vector<Geometry> geoms;
	std::vector<Light> lights;
	std::vector<Face> faces;
	std::string warnings;
};

struct ParseError {
	std::string msg;
};
struct MathError {
	std::string msg;
};

// RTIParser(scene).parseFile(path): throws ParseError / MathError.
void parse_rti_file(Scene& scene, const std::string& path);

// Affine from Eigen's Transform<double,3,Affine> storage (16 doubles, column-major) and back
Affine affine_from_eigen(const double cm[16]);
void affine_to_eigen(const Affine& a, double cm[16]);
// fwd * raw for the camera corners and the lights (Transform * Vector4d in Eigen's order),
// done once here instead of the reference's lazy caches (rtbase.h:86-95, lights.h:28-33,56-61)
void apply_scene_transforms(Scene& s);

}  // namespace rtamd
