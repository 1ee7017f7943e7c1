// TEST INFRASTRUCTURE ONLY — the INTEGRATION.md §1 binding, compiled against the
// UNMODIFIED reference classes (/root/reference/src, built by `make -C oracle ref`).
//
// INTEGRATION.md §1 gives Scene::renderScene (scene.cpp:10-59) a body that describes the
// in-memory Scene (scene.h:35-38) to librtamd as an rt_scene_desc and renders it on the
// GPU.  This program holds that body verbatim as rtamd_render_scene(scene, output) and
// checks it against the reference's own Scene::renderScene on the same parsed Scene
// (the reference's RTIParser/OBJParser, options and classes, unmodified):
//
//   integration_check <reference flags: file.rti -w W -h H [--bdepth D] [--intersection-only]>
//
// prints "match <pixels>" and exits 0 when the two images are identical binary64 for
// binary64 (W*H must be a multiple of 2000: the reference's renderScene block, see
// ref_harness.cpp), 1 otherwise.  The maintainer's patch adds `friend class Scene;` to
// Camera, PointLight, DirectionalLight and Mesh (their points, directions and bounding
// boxes are private); the #define below stands in for those four lines here.
#include <Eigen/Core>
#include <Eigen/Geometry>
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>
// (every library header the reference's headers include comes first: only the
// reference's own classes see the #define)
#define private public  // == the four `friend class Scene;` lines of INTEGRATION.md §1
#include "options.h"
#include "parsers.h"
#include "scene.h"
#undef private
#include "../include/rtamd.h"

// ---- INTEGRATION.md §1 (begin) -------------------------------------------------------
static rt_xform_desc rtamd_xform(Transformable& t) {
	rt_xform_desc x;
	std::memset(&x, 0, sizeof(x));
	std::memcpy(x.fwd, t.forwardTransform().data(), sizeof(x.fwd));  // column-major 4x4
	std::memcpy(x.inv, t.inverseTransform().data(), sizeof(x.inv));
	x.det = t.transformDeterminant();
	return x;
}

// The Scene as flat arrays (views into its own objects; `geoms`/`lights` hold the records)
static rt_scene_desc rtamd_describe(Scene& sc, std::vector<rt_geometry_desc>& geoms,
                                    std::vector<rt_light_desc>& lights) {
	rt_scene_desc d;
	std::memset(&d, 0, sizeof(d));
	d.has_camera = sc.hasCamera_;
	Camera& cam = sc.camera_;
	d.camera.xf = rtamd_xform(cam);
	const Vector4d* pts[5] = {&cam.eyePoint_, &cam.lowerLeftPoint_, &cam.lowerRightPoint_, &cam.upperLeftPoint_,
	                          &cam.upperRightPoint_};
	double* dst[5] = {d.camera.eye, d.camera.lower_left, d.camera.lower_right, d.camera.upper_left,
	                  d.camera.upper_right};
	for (int k = 0; k < 5; k++) std::memcpy(dst[k], pts[k]->data(), 4 * sizeof(double));
	geoms.assign(sc.geometries_.size(), rt_geometry_desc{});
	for (size_t i = 0; i < sc.geometries_.size(); i++) {
		Geometry* g = sc.geometries_[i].get();
		rt_geometry_desc& gd = geoms[i];
		gd.xf = rtamd_xform(*g);
		const Material& m = g->material_;
		for (int k = 0; k < 3; k++) {
			gd.material.ambient[k] = m.ambientColor_[k];
			gd.material.diffuse[k] = m.diffuseColor_[k];
			gd.material.specular[k] = m.specularColor_[k];
			gd.material.reflective[k] = m.reflectiveColor_[k];
			gd.material.translucency[k] = m.translucencyColor_[k];
		}
		gd.material.specular_coefficient = m.specularCoefficient_;
		gd.material.index_of_refractivity = m.indexOfRefractivity_;
		if (Sphere* s = dynamic_cast<Sphere*>(g)) {
			gd.kind = RT_GEOM_SPHERE;
			std::memcpy(gd.center, s->center_.data(), sizeof(gd.center));
			gd.radius = s->radius_;
		} else {
			Mesh* mesh = dynamic_cast<Mesh*>(g);
			gd.kind = RT_GEOM_MESH;
			gd.faces = reinterpret_cast<const rt_face_desc*>(mesh->faces_.data());  // Mesh::Face verbatim
			gd.n_faces = static_cast<int64_t>(mesh->faces_.size());
			std::memcpy(gd.bbox_min, mesh->boundingBoxMin_.data(), sizeof(gd.bbox_min));
			std::memcpy(gd.bbox_max, mesh->boundingBoxMax_.data(), sizeof(gd.bbox_max));
		}
	}
	lights.assign(sc.lights_.size(), rt_light_desc{});
	for (size_t i = 0; i < sc.lights_.size(); i++) {
		Light* l = sc.lights_[i].get();
		rt_light_desc& ld = lights[i];
		ld.xf = rtamd_xform(*l);
		for (int k = 0; k < 3; k++) ld.color[k] = l->color_[k];
		if (PointLight* p = dynamic_cast<PointLight*>(l)) {
			ld.kind = RT_LIGHT_POINT;
			std::memcpy(ld.vec, p->point_.data(), sizeof(ld.vec));
			ld.falloff = p->falloffExponent_;
		} else if (DirectionalLight* dl = dynamic_cast<DirectionalLight*>(l)) {
			ld.kind = RT_LIGHT_DIRECTIONAL;
			std::memcpy(ld.vec, dl->direction_.data(), sizeof(ld.vec));
		} else {
			ld.kind = RT_LIGHT_AMBIENT;
		}
	}
	d.n_geometries = static_cast<int32_t>(geoms.size());
	d.n_lights = static_cast<int32_t>(lights.size());
	d.geometries = geoms.data();
	d.lights = lights.data();
	return d;
}

// The body of Scene::renderScene(output, phandler): upload, render on GPU 0 into the
// RasterImage (H x W x 3 doubles, row-major), progress from the render loop, the
// --intersection-only normalisation included (scene.cpp:50-58).
static void rtamd_render_scene(Scene& sc, Scene::RasterImage& output, Scene::ProgressHandler phandler) {
	std::vector<rt_geometry_desc> geoms;
	std::vector<rt_light_desc> lights;
	const rt_scene_desc d = rtamd_describe(sc, geoms, lights);
	rt_scene* s = nullptr;
	if (rt_scene_create_desc(&d, /*device*/ 0, &s) != RT_OK) throw std::runtime_error(rt_last_error());
	rt_render_params p;
	std::memset(&p, 0, sizeof(p));
	p.width = static_cast<int32_t>(output.cols());
	p.height = static_cast<int32_t>(output.rows());
	p.bounce_depth = programOptions.bounceDepth_;
	p.intersection_only = programOptions.intersectionOnly_;
	p.row_begin = 0;
	p.row_end = p.height;
	p.row_step = 1;
	auto progress = [](int c, int t, void* u) {
		if (u) reinterpret_cast<Scene::ProgressHandler>(u)(c, t);
	};
	const int rc = rt_render(s, &p, output.data()->data(), progress, reinterpret_cast<void*>(phandler), nullptr);
	rt_scene_destroy(s);
	if (rc == RT_ERR_MATH) throw MathException(rt_last_error());
	if (rc != RT_OK) throw std::runtime_error(rt_last_error());
}
// ---- INTEGRATION.md §1 (end) ---------------------------------------------------------

int main(int argc, char* argv[]) {
	if (!programOptions.parseCommandLine(argc, argv)) return 2;
	Scene scene;
	for (const std::string& fn : programOptions.inputFilenames_) {
		RTIParser parser(scene);
		try {
			parser.parseFile(fn);
		} catch (const ParseException& e) {
			std::fprintf(stderr, "Error: %s\n", e.what());
			return 2;
		}
	}
	const int rows = programOptions.renderHeight_, cols = programOptions.renderWidth_;
	if (((long)rows * cols) % 2000 != 0) {
		std::fprintf(stderr, "integration_check: W*H must be a multiple of 2000 (scene.cpp:13)\n");
		return 2;
	}
	Scene::RasterImage gpu(rows, cols), ref(rows, cols);
	try {
		rtamd_render_scene(scene, gpu, nullptr);
	} catch (const std::exception& e) {
		std::fprintf(stderr, "rtamd: %s\n", e.what());
		return 2;
	}
	scene.renderScene(ref, nullptr);  // the reference's own render loop, after the GPU's
	long diff = 0;
	for (long i = 0; i < (long)rows * cols; i++)
		if (std::memcmp(gpu(i).data(), ref(i).data(), 3 * sizeof(double)) != 0) diff++;
	if (diff) {
		std::printf("mismatch %ld of %ld pixels\n", diff, (long)rows * cols);
		return 1;
	}
	std::printf("match %ld\n", (long)rows * cols);
	return 0;
}
