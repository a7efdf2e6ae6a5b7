// scene.cpp -- Scene loading/building for the MI355X path tracer.
// Host code; see scene.h.  Reference behaviour cited per function.
#include "scene.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>

#pragma clang fp contract(off)

namespace pt {

static const float kBaseModelScale = 1000.0f;   // Config.h:16 BASE_MODEL_SCALE

// ---------------------------------------------------------------------------
// glm 0.9.6 matrix restatements (column-major, m[c*4+r])
// ---------------------------------------------------------------------------
static void m4_identity(float* m) { std::memset(m, 0, 64); m[0] = m[5] = m[10] = m[15] = 1.0f; }

// type_mat4x4.inl:686-704
static void m4_mul(const float* a, const float* b, float* out) {
    float r[16];
    for (int i = 0; i < 4; i++)
        for (int k = 0; k < 4; k++)
            r[i * 4 + k] = a[0 * 4 + k] * b[i * 4 + 0] + a[1 * 4 + k] * b[i * 4 + 1] +
                           a[2 * 4 + k] * b[i * 4 + 2] + a[3 * 4 + k] * b[i * 4 + 3];
    std::memcpy(out, r, 64);
}

// gtc/matrix_transform.inl:122-134
static void m4_scale(const float* m, const float* v, float* out) {
    float r[16];
    for (int k = 0; k < 4; k++) {
        r[0 * 4 + k] = m[0 * 4 + k] * v[0];
        r[1 * 4 + k] = m[1 * 4 + k] * v[1];
        r[2 * 4 + k] = m[2 * 4 + k] * v[2];
        r[3 * 4 + k] = m[3 * 4 + k];
    }
    std::memcpy(out, r, 64);
}

// gtc/matrix_transform.inl:39-48
static void m4_translate(const float* m, const float* v, float* out) {
    float r[16];
    std::memcpy(r, m, 64);
    for (int k = 0; k < 4; k++)
        r[3 * 4 + k] = m[0 * 4 + k] * v[0] + m[1 * 4 + k] * v[1] + m[2 * 4 + k] * v[2] + m[3 * 4 + k];
    std::memcpy(out, r, 64);
}

// gtc/matrix_transform.inl:51-85
static void m4_rotate(const float* m, float angle, f3 axis_in, float* out) {
    float c = std::cos(angle), s = std::sin(angle);
    f3 axis = normalize(axis_in);
    f3 temp = axis * (1.0f - c);
    float R[3][3];
    R[0][0] = c + temp.x * axis.x;
    R[0][1] = 0 + temp.x * axis.y + s * axis.z;
    R[0][2] = 0 + temp.x * axis.z - s * axis.y;
    R[1][0] = 0 + temp.y * axis.x - s * axis.z;
    R[1][1] = c + temp.y * axis.y;
    R[1][2] = 0 + temp.y * axis.z + s * axis.x;
    R[2][0] = 0 + temp.z * axis.x + s * axis.y;
    R[2][1] = 0 + temp.z * axis.y - s * axis.x;
    R[2][2] = c + temp.z * axis.z;
    float r[16];
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 4; k++)
            r[i * 4 + k] = m[0 * 4 + k] * R[i][0] + m[1 * 4 + k] * R[i][1] + m[2 * 4 + k] * R[i][2];
    for (int k = 0; k < 4; k++) r[3 * 4 + k] = m[3 * 4 + k];
    std::memcpy(out, r, 64);
}

// detail::compute_inverse<tmat4x4> (type_mat4x4.inl:37-92)
static void m4_inverse(const float* mm, float* out) {
    auto M = [&](int c, int r) { return mm[c * 4 + r]; };
    float C00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
    float C02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
    float C03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
    float C04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
    float C06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
    float C07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
    float C08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
    float C10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
    float C11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
    float C12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
    float C14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
    float C15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
    float C16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
    float C18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
    float C19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
    float C20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
    float C22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
    float C23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
    const float F0[4] = {C00, C00, C02, C03}, F1[4] = {C04, C04, C06, C07}, F2[4] = {C08, C08, C10, C11};
    const float F3[4] = {C12, C12, C14, C15}, F4[4] = {C16, C16, C18, C19}, F5[4] = {C20, C20, C22, C23};
    const float V0[4] = {M(1, 0), M(0, 0), M(0, 0), M(0, 0)};
    const float V1[4] = {M(1, 1), M(0, 1), M(0, 1), M(0, 1)};
    const float V2[4] = {M(1, 2), M(0, 2), M(0, 2), M(0, 2)};
    const float V3[4] = {M(1, 3), M(0, 3), M(0, 3), M(0, 3)};
    float I0[4], I1[4], I2[4], I3[4];
    for (int k = 0; k < 4; k++) {
        I0[k] = V1[k] * F0[k] - V2[k] * F1[k] + V3[k] * F2[k];
        I1[k] = V0[k] * F0[k] - V2[k] * F3[k] + V3[k] * F4[k];
        I2[k] = V0[k] * F1[k] - V1[k] * F3[k] + V3[k] * F5[k];
        I3[k] = V0[k] * F2[k] - V1[k] * F4[k] + V2[k] * F5[k];
    }
    const float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
    float inv[16];
    for (int k = 0; k < 4; k++) {
        inv[0 * 4 + k] = I0[k] * SA[k];
        inv[1 * 4 + k] = I1[k] * SB[k];
        inv[2 * 4 + k] = I2[k] * SA[k];
        inv[3 * 4 + k] = I3[k] * SB[k];
    }
    const float row0[4] = {inv[0], inv[4], inv[8], inv[12]};
    float d0[4];
    for (int k = 0; k < 4; k++) d0[k] = M(0, k) * row0[k];
    float d1 = (d0[0] + d0[1]) + (d0[2] + d0[3]);
    float od = 1.0f / d1;
    for (int i = 0; i < 16; i++) out[i] = inv[i] * od;
}

void model_matrices(const float scale[3], const float rot_deg[3], const float translate[3],
                    float m2w[16], float w2m[16]) {
    float I[16], S[16], R[16], T[16], TR[16];
    m4_identity(I);
    m4_scale(I, scale, S);
    const float deg2rad = (float)0.01745329251994329576923690768489;  // glm::radians
    m4_rotate(I, rot_deg[0] * deg2rad, mk3(1.0f, 0.0f, 0.0f), R);
    m4_rotate(R, rot_deg[1] * deg2rad, mk3(0.0f, 1.0f, 0.0f), R);
    m4_rotate(R, rot_deg[2] * deg2rad, mk3(0.0f, 0.0f, 1.0f), R);
    m4_translate(I, translate, T);
    m4_mul(T, R, TR);
    m4_mul(TR, S, m2w);
    m4_inverse(m2w, w2m);
}

// detail::compute_inverse<tmat3x3> (type_mat3x3.inl:37-56) of mat3(m): out[c*3+r] = Inverse[c][r]
static void m3_inverse_of_m4(const float* m, float* out) {
    auto M = [&](int c, int r) { return m[c * 4 + r]; };
    float od = 1.0f / (+M(0, 0) * (M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2))
                       - M(1, 0) * (M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2))
                       + M(2, 0) * (M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2)));
    out[0 * 3 + 0] = +(M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) * od;
    out[1 * 3 + 0] = -(M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2)) * od;
    out[2 * 3 + 0] = +(M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1)) * od;
    out[0 * 3 + 1] = -(M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) * od;
    out[1 * 3 + 1] = +(M(0, 0) * M(2, 2) - M(2, 0) * M(0, 2)) * od;
    out[2 * 3 + 1] = -(M(0, 0) * M(2, 1) - M(2, 0) * M(0, 1)) * od;
    out[0 * 3 + 2] = +(M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2)) * od;
    out[1 * 3 + 2] = -(M(0, 0) * M(1, 2) - M(1, 0) * M(0, 2)) * od;
    out[2 * 3 + 2] = +(M(0, 0) * M(1, 1) - M(1, 0) * M(0, 1)) * od;
}

// ---------------------------------------------------------------------------
// Mesh loading
// ---------------------------------------------------------------------------

// Appends one aiMesh worth of data exactly like Scene::processMesh
// (Scene.cpp:264-291): positions/normals scaled by BASE_MODEL_SCALE, bbox
// updated per vertex, triangle indices offset by the mesh's first vertex.
int Scene::addVertexRun(const std::vector<f3>& pos, const std::vector<f3>& nrm, const std::vector<int>& tri_local) {
    Mesh mesh;
    mesh.vertex_indices.start_index = (int)vertices.size();
    for (size_t i = 0; i < pos.size(); i++) {
        Vertex v;
        v.position = mk3(pos[i].x * kBaseModelScale, pos[i].y * kBaseModelScale, pos[i].z * kBaseModelScale);
        v.normal = mk3(nrm[i].x * kBaseModelScale, nrm[i].y * kBaseModelScale, nrm[i].z * kBaseModelScale);
        vertices.push_back(v);
        mesh.bounding_box.update(v.position);
    }
    mesh.vertex_indices.end_index = (int)vertices.size();
    mesh.triangle_indices.start_index = (int)triangles.size();
    for (size_t i = 0; i + 2 < tri_local.size(); i += 3) {
        Triangle t;
        for (int j = 0; j < 3; j++) t.vertex_indices[j] = mesh.vertex_indices.start_index + tri_local[i + j];
        triangles.push_back(t);
    }
    mesh.triangle_indices.end_index = (int)triangles.size();
    meshes.push_back(mesh);
    built = false;
    return (int)meshes.size() - 1;
}

static f3 geo_normal(f3 p0, f3 p1, f3 p2) { return normalize(cross(p1 - p0, p2 - p0)); }

// Scene::loadAndProcessMeshFile (Scene.cpp:226-238) with Assimp's OBJ importer
// semantics as the reference invokes it (aiProcess_FlipUVs only): every face
// corner becomes its own vertex (no JoinIdenticalVertices), one aiMesh per
// file.  Decimal -> double -> float.  Extensions: polygons fan-triangulated,
// corners without `vn` get the face's geometric normal.
int Scene::loadObj(const std::string& path) {
    std::ifstream in(path);
    if (!in) { last_error = "Error loading mesh: cannot open " + path; return -1; }
    std::vector<f3> V, N, pos, nrm;
    std::vector<int> tri;
    std::string line;
    int base = 0;
    std::vector<std::pair<int, int>> corners;
    while (std::getline(in, line)) {
        if (line.size() < 2) continue;
        const char* s = line.c_str();
        if (s[0] == 'v' && s[1] == ' ') {
            char* e;
            double x = std::strtod(s + 2, &e), y = std::strtod(e, &e), z = std::strtod(e, &e);
            V.push_back(mk3((float)x, (float)y, (float)z));
        } else if (s[0] == 'v' && s[1] == 'n' && (s[2] == ' ' || s[2] == '\t')) {
            char* e;
            double x = std::strtod(s + 3, &e), y = std::strtod(e, &e), z = std::strtod(e, &e);
            N.push_back(mk3((float)x, (float)y, (float)z));
        } else if (s[0] == 'f' && (s[1] == ' ' || s[1] == '\t')) {
            corners.clear();
            std::istringstream ss(line.substr(2));
            std::string tok;
            while (ss >> tok) {
                int vi = 0, ni = 0;
                bool has_n = false;
                size_t p1 = tok.find('/');
                vi = std::atoi(tok.substr(0, p1).c_str());
                if (p1 != std::string::npos) {
                    size_t p2 = tok.find('/', p1 + 1);
                    if (p2 != std::string::npos && p2 + 1 < tok.size()) {
                        ni = std::atoi(tok.substr(p2 + 1).c_str());
                        has_n = true;
                    }
                }
                vi = vi > 0 ? vi - 1 : (int)V.size() + vi;
                if (has_n) ni = ni > 0 ? ni - 1 : (int)N.size() + ni;
                if (vi < 0 || vi >= (int)V.size() || (has_n && (ni < 0 || ni >= (int)N.size()))) {
                    last_error = "Error loading mesh: bad face index in " + path;
                    return -1;
                }
                corners.push_back({vi, has_n ? ni : -1});
            }
            int k = (int)corners.size();
            if (k < 3) continue;
            bool need_geo = false;
            for (auto& c : corners) need_geo |= (c.second < 0);
            f3 g = need_geo ? geo_normal(V[corners[0].first], V[corners[1].first], V[corners[2].first]) : mk3(0, 0, 0);
            for (int j = 0; j < k; j++) {
                pos.push_back(V[corners[j].first]);
                nrm.push_back(corners[j].second >= 0 ? N[corners[j].second] : g);
            }
            for (int j = 1; j + 1 < k; j++) {
                tri.push_back(base);
                tri.push_back(base + j);
                tri.push_back(base + j + 1);
            }
            base += k;
        }
    }
    return addVertexRun(pos, nrm, tri);
}

int Scene::addMesh(const float* p, const float* n, int nv, const int* tris, int nt) {
    std::vector<f3> pos(nv), nrm(nv);
    for (int i = 0; i < nv; i++) {
        pos[i] = mk3(p[3 * i], p[3 * i + 1], p[3 * i + 2]);
        nrm[i] = mk3(n[3 * i], n[3 * i + 1], n[3 * i + 2]);
    }
    std::vector<int> t(tris, tris + 3 * (size_t)nt);
    for (int v : t)
        if (v < 0 || v >= nv) { last_error = "addMesh: triangle index out of range"; return -1; }
    return addVertexRun(pos, nrm, t);
}

int Scene::addModel(int mesh_index, const float scale[3], const float rot_deg[3], const float translate[3],
                    int material_type, const float color[3]) {
    if (mesh_index < 0 || mesh_index >= (int)meshes.size()) { last_error = "addModel: bad mesh index"; return -1; }
    if (material_type < MAT_DIFFUSE || material_type > MAT_METAL) { last_error = "addModel: bad material"; return -1; }
    Model m;
    m.mesh_index = mesh_index;
    model_matrices(scale, rot_deg, translate, m.model_to_world, m.world_to_model);
    m.mat.material_type = material_type;
    for (int i = 0; i < 3; i++) m.mat.color[i] = color[i];
    models.push_back(m);
    built = false;
    return (int)models.size() - 1;
}

// ---------------------------------------------------------------------------
// Config.txt grammar (PathTracerAP/Config.txt): blank-line separated blocks,
// first line = keyword.  See DESIGN.md "Scene description".
// ---------------------------------------------------------------------------
static std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) a++;
    while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

static bool parse_vec(const std::string& s, std::vector<double>& out) {
    size_t a = s.find('['), b = s.find(']');
    if (a == std::string::npos || b == std::string::npos || b < a) return false;
    out.clear();
    std::string body = s.substr(a + 1, b - a - 1);
    std::stringstream ss(body);
    std::string tok;
    while (std::getline(ss, tok, ',')) {
        tok = trim(tok);
        if (tok.empty()) return false;
        char* e;
        double v = std::strtod(tok.c_str(), &e);
        if (*e != '\0') return false;
        out.push_back(v);
    }
    return true;
}

static int material_from_name(const std::string& k) {
    if (k == "DIFFUSE") return MAT_DIFFUSE;
    if (k == "SPECULAR") return MAT_SPECULAR;
    if (k == "REFLECTIVE") return MAT_REFLECTIVE;
    if (k == "REFRACTIVE" || k == "REFRACRIVE") return MAT_REFRACTIVE;  // Config.txt:29 spelling
    if (k == "EMISSIVE") return MAT_EMISSIVE;
    if (k == "COAT") return MAT_COAT;
    if (k == "METAL") return MAT_METAL;
    return -1;
}

// Generated primitives for the Config.txt SPHERE / BOX blocks (in OBJ units,
// i.e. before BASE_MODEL_SCALE, like a loaded file).
static void gen_box(const double* mx, const double* mn, std::vector<f3>& pos, std::vector<f3>& nrm, std::vector<int>& tri) {
    const float lo[3] = {(float)mn[0], (float)mn[1], (float)mn[2]};
    const float hi[3] = {(float)mx[0], (float)mx[1], (float)mx[2]};
    for (int axis = 0; axis < 3; axis++)
        for (int side = 0; side < 2; side++) {
            int u = (axis + 1) % 3, v = (axis + 2) % 3;
            float n[3] = {0, 0, 0};
            n[axis] = side ? 1.0f : -1.0f;
            float c[4][3];
            const int uv[4][2] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
            for (int q = 0; q < 4; q++) {
                c[q][axis] = side ? hi[axis] : lo[axis];
                c[q][u] = uv[q][0] ? hi[u] : lo[u];
                c[q][v] = uv[q][1] ? hi[v] : lo[v];
            }
            int b = (int)pos.size();
            for (int q = 0; q < 4; q++) {
                pos.push_back(mk3(c[q][0], c[q][1], c[q][2]));
                nrm.push_back(mk3(n[0], n[1], n[2]));
            }
            if (side) { tri.insert(tri.end(), {b, b + 1, b + 2, b, b + 2, b + 3}); }
            else { tri.insert(tri.end(), {b, b + 2, b + 1, b, b + 3, b + 2}); }
        }
}

static void gen_sphere(double radius, const double* ctr, std::vector<f3>& pos, std::vector<f3>& nrm, std::vector<int>& tri) {
    const int NU = 48, NV = 24;
    for (int j = 0; j <= NV; j++)
        for (int i = 0; i <= NU; i++) {
            double th = M_PI * j / NV, ph = 2 * M_PI * i / NU;
            double nx = std::sin(th) * std::cos(ph), ny = std::cos(th), nz = std::sin(th) * std::sin(ph);
            pos.push_back(mk3((float)(ctr[0] + radius * nx), (float)(ctr[1] + radius * ny), (float)(ctr[2] + radius * nz)));
            nrm.push_back(mk3((float)nx, (float)ny, (float)nz));
        }
    for (int j = 0; j < NV; j++)
        for (int i = 0; i < NU; i++) {
            int a = j * (NU + 1) + i, b = a + NU + 1;
            if (j != 0) tri.insert(tri.end(), {a, a + 1, b});
            if (j != NV - 1) tri.insert(tri.end(), {a + 1, b + 1, b});
        }
}

int Scene::loadConfig(const std::string& path) {
    std::ifstream in(path);
    if (!in) { last_error = "cannot open scene config " + path; return -1; }
    std::string dir = ".";
    size_t sl = path.find_last_of('/');
    if (sl != std::string::npos) dir = path.substr(0, sl);
    std::vector<std::vector<std::string>> blocks;
    std::vector<std::string> cur;
    std::string line;
    while (std::getline(in, line)) {
        std::string t = trim(line);
        size_t hash = t.find('#');
        if (hash == 0) continue;
        if (t.rfind("//", 0) == 0) continue;   // Config.txt:18 comment style
        if (t.empty()) {
            if (!cur.empty()) { blocks.push_back(cur); cur.clear(); }
            continue;
        }
        cur.push_back(t);
    }
    if (!cur.empty()) blocks.push_back(cur);

    struct Mat { int type; float color[3]; };
    std::map<std::string, Mat> mats;
    std::map<std::string, int> named_mesh;   // OBJ name or path -> mesh index
    auto resolve = [&](const std::string& p) { return (!p.empty() && p[0] == '/') ? p : dir + "/" + p; };
    auto fail = [&](const std::string& msg) { last_error = path + ": " + msg; return -2; };

    for (auto& b : blocks) {
        const std::string& kw = b[0];
        int mt = material_from_name(kw);
        if (mt >= 0) {
            if (b.size() < 3) return fail("material block needs name and [r,g,b]");
            std::vector<double> c;
            if (!parse_vec(b[2], c) || c.size() != 3) return fail("bad material color " + b[2]);
            Mat m; m.type = mt;
            for (int i = 0; i < 3; i++) m.color[i] = (float)c[i];
            mats[b[1]] = m;
        }
    }
    for (auto& b : blocks) {
        const std::string& kw = b[0];
        if (material_from_name(kw) >= 0) continue;
        if (kw == "RENDER") {
            for (size_t i = 1; i < b.size(); i++) {
                std::string key = b[i].substr(0, b[i].find(':'));
                std::string val = b[i].find(':') == std::string::npos ? "" : trim(b[i].substr(b[i].find(':') + 1));
                std::vector<double> v;
                if (key == "resolution" && parse_vec(val, v) && v.size() == 2) {
                    settings.width = (int)v[0]; settings.height = (int)v[1]; settings.has_width = true;
                } else if (key == "iterations") { settings.iterations = std::atoi(val.c_str()); settings.has_iterations = true; }
                else if (key == "bounces") { settings.max_bounces = std::atoi(val.c_str()); settings.has_bounces = true; }
                else if (key == "grid" && parse_vec(val, v) && v.size() == 3) {
                    for (int k = 0; k < 3; k++) settings.grid[k] = (int)v[k];
                } else if (key == "accel") {
                    settings.accel = (val == "bvh") ? ACCEL_BVH : (val == "grid_fast") ? ACCEL_GRID_FAST : ACCEL_GRID;
                    settings.has_accel = true;
                } else return fail("bad RENDER line " + b[i]);
            }
            continue;
        }
        if (kw == "OBJ") {
            if (b.size() < 3) return fail("OBJ block needs name and path");
            int m = loadObj(resolve(b[2]));
            if (m < 0) return -3;
            named_mesh[b[1]] = m;
            continue;
        }
        if (kw != "MESH" && kw != "SPHERE" && kw != "BOX") return fail("unknown block " + kw);
        if (b.size() < 2) return fail(kw + " block needs a name");
        int mesh = -1;
        size_t first_attr = 2;
        if (kw == "MESH") {
            if (b.size() < 3) return fail("MESH block needs an obj path or OBJ name");
            auto it = named_mesh.find(b[2]);
            if (it != named_mesh.end()) mesh = it->second;
            else {
                mesh = loadObj(resolve(b[2]));
                if (mesh < 0) return -3;
                named_mesh[b[2]] = mesh;
            }
            first_attr = 3;
        } else if (kw == "BOX") {          // Config.txt:9-15: BOX name [max] [min]
            std::vector<double> mx, mn;
            if (b.size() < 4 || !parse_vec(b[2], mx) || !parse_vec(b[3], mn) || mx.size() != 3 || mn.size() != 3)
                return fail("BOX needs [max] and [min]");
            std::vector<f3> pos, nrm; std::vector<int> tri;
            gen_box(mx.data(), mn.data(), pos, nrm, tri);
            mesh = addVertexRun(pos, nrm, tri);
            first_attr = 4;
        } else {                           // Config.txt:1-7: SPHERE name radius [center]
            std::vector<double> c;
            if (b.size() < 4 || !parse_vec(b[3], c) || c.size() != 3) return fail("SPHERE needs radius and [center]");
            std::vector<f3> pos, nrm; std::vector<int> tri;
            gen_sphere(std::atof(b[2].c_str()), c.data(), pos, nrm, tri);
            mesh = addVertexRun(pos, nrm, tri);
            first_attr = 4;
        }
        float scale[3] = {1, 1, 1}, rot[3] = {0, 0, 0}, tr[3] = {0, 0, 0};
        Mat mat; mat.type = MAT_DIFFUSE; mat.color[0] = mat.color[1] = mat.color[2] = 0.98f;
        for (size_t i = first_attr; i < b.size(); i++) {
            std::string key = b[i].substr(0, b[i].find(':'));
            std::string val = b[i].find(':') == std::string::npos ? "" : trim(b[i].substr(b[i].find(':') + 1));
            std::vector<double> v;
            if (key == "material") {
                auto it = mats.find(val);
                if (it == mats.end()) return fail("unknown material " + val);
                mat = it->second;
                continue;
            }
            if (!parse_vec(val, v) || v.size() != 3) return fail("bad attribute " + b[i]);
            float f[3] = {(float)v[0], (float)v[1], (float)v[2]};
            if (key == "translate") std::memcpy(tr, f, sizeof f);
            else if (key == "scale") std::memcpy(scale, f, sizeof f);
            else if (key == "rotate" || key == "rotateX") std::memcpy(rot, f, sizeof f);  // Config.txt:6 "rotateX:[x,y,z]"
            else return fail("unknown attribute " + key);
        }
        if (addModel(mesh, scale, rot, tr, mat.type, mat.color) < 0) return -4;
    }
    if (models.empty()) return fail("scene has no MESH/BOX/SPHERE instances");
    return 0;
}

// ---------------------------------------------------------------------------
// addMeshesToGrid (Scene.cpp:293-396)
// ---------------------------------------------------------------------------
void Scene::addMeshesToGrid() {
    grids.clear();
    voxels.clear();
    per_voxel_data_pool.clear();
    tri_vbox.assign(triangles.size() * 2, 0);
    const int GX = grid_dim[0], GY = grid_dim[1], GZ = grid_dim[2];
    std::vector<bool> is_mesh_processed(meshes.size(), false);
    std::vector<int> grid_index_cache(meshes.size(), 0);
    for (size_t i = 0; i < models.size(); i++) {
        int mi = models[i].mesh_index;
        if (is_mesh_processed[mi]) { models[i].grid_index = grid_index_cache[mi]; continue; }
        is_mesh_processed[mi] = true;
        grid_index_cache[mi] = (int)grids.size();
        models[i].grid_index = (int)grids.size();
        Grid grid;
        grid.entity_type = ENTITY_MODEL;
        grid.entity_index = (int)i;
        const BoundingBox& bb = meshes[mi].bounding_box;
        std::vector<std::vector<int>> buf((size_t)GX * GY * GZ);
        grid.voxel_width[0] = (bb.max.x - bb.min.x) / (float)GX;
        grid.voxel_width[1] = (bb.max.y - bb.min.y) / (float)GY;
        grid.voxel_width[2] = (bb.max.z - bb.min.z) / (float)GZ;
        const float bmin[3] = {bb.min.x, bb.min.y, bb.min.z};
        const int gd[3] = {GX, GY, GZ};
        for (int t = meshes[mi].triangle_indices.start_index; t < meshes[mi].triangle_indices.end_index; t++) {
            // computeVoxelIndex (Scene.cpp:293-316)
            BoundingBox tb;
            for (int j = 0; j < 3; j++) tb.update(vertices[triangles[t].vertex_indices[j]].position);
            const float tmin[3] = {tb.min.x, tb.min.y, tb.min.z}, tmax[3] = {tb.max.x, tb.max.y, tb.max.z};
            int mn[3], mx[3];
            for (int a = 0; a < 3; a++) {
                mn[a] = f2i_x86(std::floor(std::fabs(bmin[a] - tmin[a]) / grid.voxel_width[a]));
                mx[a] = f2i_x86(std::floor(std::fabs(bmin[a] - tmax[a]) / grid.voxel_width[a]));
                mn[a] = mn[a] < 0 ? 0 : (mn[a] > gd[a] - 1 ? gd[a] - 1 : mn[a]);
                mx[a] = mx[a] < 0 ? 0 : (mx[a] > gd[a] - 1 ? gd[a] - 1 : mx[a]);
            }
            // the voxel box [mn, mx] is exactly the set of voxels whose list holds t
            tri_vbox[2 * (size_t)t] = mn[0] | (mn[1] << 10) | (mn[2] << 20);
            tri_vbox[2 * (size_t)t + 1] = mx[0] | (mx[1] << 10) | (mx[2] << 20);
            for (int z = mn[2]; z <= mx[2]; z++)
                for (int y = mn[1]; y <= mx[1]; y++)
                    for (int x = mn[0]; x <= mx[0]; x++) buf[(size_t)x + (size_t)y * GX + (size_t)GX * GY * z].push_back(t);
        }
        grid.voxelIndices.start_index = (int)voxels.size();
        for (auto& v : buf) {
            Voxel vx;
            vx.entity_type = ENTITY_TRIANGLE;
            vx.entity_index_range.start_index = (int)per_voxel_data_pool.size();
            per_voxel_data_pool.insert(per_voxel_data_pool.end(), v.begin(), v.end());
            vx.entity_index_range.end_index = (int)per_voxel_data_pool.size();
            voxels.push_back(vx);
        }
        grid.voxelIndices.end_index = (int)voxels.size();
        grids.push_back(grid);
    }
}

void Scene::buildDeviceTables() {
    const size_t nt = triangles.size();
    tri_geom.assign(nt * 12, 0.0f);
    tri_normal.assign(nt * 4, 0.0f);
    for (size_t t = 0; t < nt; t++) {
        const Vertex& a = vertices[triangles[t].vertex_indices[0]];
        const Vertex& b = vertices[triangles[t].vertex_indices[1]];
        const Vertex& c = vertices[triangles[t].vertex_indices[2]];
        // computeRayTriangleIntersection (Renderer.cpp:183-184): v0v1, v0v2
        f3 e1 = b.position - a.position, e2 = c.position - a.position;
        float* g = &tri_geom[t * 12];
        g[0] = a.position.x; g[1] = a.position.y; g[2] = a.position.z;
        g[4] = e1.x; g[5] = e1.y; g[6] = e1.z;
        g[8] = e2.x; g[9] = e2.y; g[10] = e2.z;
        // Renderer.cpp:203: normalize((n0 + n1 + n2) * (1/3.0f))
        f3 n = normalize(((a.normal + b.normal) + c.normal) * (1 / 3.0f));
        float* q = &tri_normal[t * 4];
        q[0] = n.x; q[1] = n.y; q[2] = n.z; q[3] = 0.0f;
    }
    bvh_tri_geom.assign(bvh_tri_order.size() * 12, 0.0f);
    for (size_t i = 0; i < bvh_tri_order.size(); i++) {
        const int t = bvh_tri_order[i];
        std::memcpy(&bvh_tri_geom[i * 12], &tri_geom[(size_t)t * 12], 12 * sizeof(float));
        std::memcpy(&bvh_tri_geom[i * 12 + 3], &t, sizeof(int));
        std::memcpy(&bvh_tri_geom[i * 12 + 7], &tri_vbox[2 * (size_t)t], sizeof(int));
        std::memcpy(&bvh_tri_geom[i * 12 + 11], &tri_vbox[2 * (size_t)t + 1], sizeof(int));
    }
    model_recs.resize(models.size());
    model_shade.resize(models.size());
    for (size_t i = 0; i < models.size(); i++) {
        const Model& m = models[i];
        ModelRec& r = model_recs[i];
        std::memset(&r, 0, sizeof r);
        for (int c = 0; c < 4; c++)
            for (int k = 0; k < 3; k++) {
                r.w2m[c * 3 + k] = m.world_to_model[c * 4 + k];
                r.m2w[c * 3 + k] = m.model_to_world[c * 4 + k];
            }
        m3_inverse_of_m4(m.model_to_world, r.nm);
        const Mesh& mesh = meshes[m.mesh_index];
        r.bbox[0] = mesh.bounding_box.min.x; r.bbox[1] = mesh.bounding_box.min.y; r.bbox[2] = mesh.bounding_box.min.z;
        r.bbox[3] = mesh.bounding_box.max.x; r.bbox[4] = mesh.bounding_box.max.y; r.bbox[5] = mesh.bounding_box.max.z;
        const Grid& g = grids[m.grid_index];
        // computeRayGridIntersection uses models[grid.entity_index]'s mesh bbox == this mesh's.
        for (int k = 0; k < 3; k++) r.vw[k] = g.voxel_width[k];
        r.vox_start = g.voxelIndices.start_index;
        r.leaf_base = mesh_leaf_base.empty() ? 0 : mesh_leaf_base[m.mesh_index];
        r.tri_start = mesh.triangle_indices.start_index;
        r.tri_end = mesh.triangle_indices.end_index;
        r.bvh_root = mesh_bvh_root.empty() ? -1 : mesh_bvh_root[m.mesh_index];
        r.bvh4_root = mesh_bvh4_root.empty() ? -1 : mesh_bvh4_root[m.mesh_index];
        ModelShade& sh = model_shade[i];
        for (int k = 0; k < 3; k++) sh.color[k] = m.mat.color[k];
        sh.mat_type = m.mat.material_type;
        world_box(m, mesh, r.bvh_root, r.wbox);
        // Bounded hit-set collection (ACCEL_GRID_FAST).  A member h whose voxel box the
        // DDA enters at ray parameter tau has its hit within tau + R_h, R_h = the diameter
        // of its voxel box grown by the test's tolerance region (<= 1% of the triangle's
        // bbox diagonal outside the bbox on each side) and the DDA's +EPSILON index shift.
        // reach = max_h R_h (+2% and a rounding slack); wdelta = the tier-1 window.
        double rmax = 0;
        for (int t = mesh.triangle_indices.start_index; t < mesh.triangle_indices.end_index; t++) {
            BoundingBox tb;
            for (int j = 0; j < 3; j++) tb.update(vertices[triangles[t].vertex_indices[j]].position);
            const double dx = (double)tb.max.x - tb.min.x, dy = (double)tb.max.y - tb.min.y, dz = (double)tb.max.z - tb.min.z;
            const double tdiag = std::sqrt(dx * dx + dy * dy + dz * dz);
            const int lo = tri_vbox[2 * (size_t)t], hi = tri_vbox[2 * (size_t)t + 1];
            double vb = 0;
            for (int k = 0; k < 3; k++) {
                const double n = (double)(((hi >> (10 * k)) & 1023) - ((lo >> (10 * k)) & 1023) + 1);
                vb += (n * g.voxel_width[k]) * (n * g.voxel_width[k]);
            }
            rmax = std::max(rmax, std::sqrt(vb) + 0.02 * tdiag + 4.0 * (double)kEps);
        }
        const double vd = std::sqrt((double)g.voxel_width[0] * g.voxel_width[0] + (double)g.voxel_width[1] * g.voxel_width[1] +
                                    (double)g.voxel_width[2] * g.voxel_width[2]);
        const double bd = vd * std::sqrt((double)grid_dim[0] * grid_dim[0] + (double)grid_dim[1] * grid_dim[1] +
                                         (double)grid_dim[2] * grid_dim[2]) / std::sqrt(3.0);
        const double R = 1.02 * rmax + 1e-4 * bd + 1e-3;
        r.reach = std::isfinite(R) ? (float)R : 3e38f;
        const double W = 0.05 * vd + 1e-4 * bd + 1e-3;
        r.wdelta = std::isfinite(W) ? (float)W : 3e38f;
        // Walk certificate (renderer.hip walk_certify): position slack that covers the
        // DDA's +EPSILON initial-index shift and the rounding of its crossing
        // parameters (<= 26 rounded adds of positive steps, plus the initial
        // (boundary - pt) * inv) relative to the exact ray, per axis.
        for (int k = 0; k < 3; k++) {
            r.ivw[k] = (float)(1.0 / (double)g.voxel_width[k]);
            const double span = (double)g.voxel_width[k] * grid_dim[k];
            const double mag = std::fabs((double)r.bbox[k]) + std::fabs((double)r.bbox[k + 3]) + span;
            r.cslack[k] = (float)(2.0 * kEps + 4.8e-7 * (grid_dim[k] + 4) * mag);
        }
    }
}

// Conservative world AABB of an instance (instance culling in the kernels):
// the mesh bbox united with every triangle grown by the reference test's
// barycentric tolerances (all points the test can accept), grown by 1e-3 of
// the diagonal, mapped through model_to_world in double and padded again.  A
// ray that misses it cannot pass the reference's slab test, and no hit the
// test accepts lies outside it.
void Scene::world_box(const Model& m, const Mesh& mesh, int root, float* out) const {
    (void)root;
    double lo[3] = {mesh.bounding_box.min.x, mesh.bounding_box.min.y, mesh.bounding_box.min.z};
    double hi[3] = {mesh.bounding_box.max.x, mesh.bounding_box.max.y, mesh.bounding_box.max.z};
    // every point the reference triangle test can accept: u >= -e, v >= -e, u + v <= 1 + e
    const double e = (double)kEps;
    const double uv[3][2] = {{-e, -e}, {1 + 2 * e, -e}, {-e, 1 + 2 * e}};
    for (int t = mesh.triangle_indices.start_index; t < mesh.triangle_indices.end_index; t++) {
        const f3 a = vertices[triangles[t].vertex_indices[0]].position;
        const f3 b = vertices[triangles[t].vertex_indices[1]].position;
        const f3 c = vertices[triangles[t].vertex_indices[2]].position;
        const double v0[3] = {a.x, a.y, a.z};
        const double e1[3] = {(double)b.x - a.x, (double)b.y - a.y, (double)b.z - a.z};
        const double e2[3] = {(double)c.x - a.x, (double)c.y - a.y, (double)c.z - a.z};
        for (int q = 0; q < 3; q++)
            for (int k = 0; k < 3; k++) {
                const double pk = v0[k] + uv[q][0] * e1[k] + uv[q][1] * e2[k];
                lo[k] = std::min(lo[k], pk);
                hi[k] = std::max(hi[k], pk);
            }
    }
    double diag = 0;
    for (int k = 0; k < 3; k++) diag += (hi[k] - lo[k]) * (hi[k] - lo[k]);
    diag = std::sqrt(std::max(diag, 0.0));
    const double pad = 1e-3 * diag + 1.0;
    double wlo[3] = {1e300, 1e300, 1e300}, whi[3] = {-1e300, -1e300, -1e300};
    bool finite = std::isfinite(diag);
    for (int c = 0; c < 8; c++) {
        const double p[3] = {(c & 1) ? hi[0] + pad : lo[0] - pad, (c & 2) ? hi[1] + pad : lo[1] - pad,
                             (c & 4) ? hi[2] + pad : lo[2] - pad};
        for (int k = 0; k < 3; k++) {
            const double w = (double)m.model_to_world[0 * 4 + k] * p[0] + (double)m.model_to_world[1 * 4 + k] * p[1] +
                             (double)m.model_to_world[2 * 4 + k] * p[2] + (double)m.model_to_world[3 * 4 + k];
            finite &= std::isfinite(w);
            wlo[k] = std::min(wlo[k], w);
            whi[k] = std::max(whi[k], w);
        }
    }
    double wd = 0;
    for (int k = 0; k < 3; k++) wd += (whi[k] - wlo[k]) * (whi[k] - wlo[k]);
    const double wpad = 1e-4 * std::sqrt(std::max(wd, 0.0)) + 1e-2;
    for (int k = 0; k < 3; k++) {
        out[k] = finite ? (float)(wlo[k] - wpad) : -3e38f;
        out[3 + k] = finite ? (float)(whi[k] + wpad) : 3e38f;
    }
}

int Scene::build(const int gd[3], bool with_bvh) {
    for (int k = 0; k < 3; k++) {
        if (gd[k] <= 0 || gd[k] > 1024) { last_error = "grid dimensions must be in [1,1024]"; return -1; }
        grid_dim[k] = gd[k];
    }
    if (models.empty()) { last_error = "scene has no models"; return -1; }
    addMeshesToGrid();
    bvh_nodes.clear();
    bvh_tri_order.clear();
    mesh_bvh_root.assign(meshes.size(), -1);
    if (with_bvh)
        for (size_t m = 0; m < meshes.size(); m++) buildBvh((int)m);
    buildBvh4();
    buildDeviceTables();
    built = true;
    return 0;
}

int Scene::ensureBvh() {
    if (!built) { last_error = "scene not built (call build first)"; return -1; }
    if (!bvh_nodes.empty()) return 0;
    const int gd[3] = {grid_dim[0], grid_dim[1], grid_dim[2]};
    return build(gd, true);        // the same grid again (deterministic), plus every mesh's BLAS
}

}  // namespace pt
