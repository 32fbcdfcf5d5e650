// Runs the reference's own CPU BSP walk -- intersect_min_max + intersect_bsp_array +
// intersect_triangle of js/bsp_tree/modules/BspTree_interleaved.js:237-352 -- under
// node, on the tree that file's build_bsp_tree (:154-234) builds, for a committed
// ray set.  Nothing from the reference is copied: Aabb.js and BspTree_interleaved.js
// are read from the directory given on the command line and evaluated in a vm
// sandbox.  What the sandbox supplies:
//   * the MV.js vector helpers those files call (vec3, vec4, subtract, cross, dot,
//     length, normalize, flatten).  MV.js -- the companion library of Angel &
//     Shreiner, "Interactive Computer Graphics" -- is not vendored in the reference;
//     its published definitions are restated below (component formulas, dot as a
//     left-to-right sum starting from 0.0);
//   * a WebGPU device stub whose createBuffer/writeBuffer do nothing;
//   * g_drawingInfo (the global the walk reads): attribs stride 8 (position at
//     0..2) and indices stride 4 (v0, v1, v2, material), i.e. the layout of
//     OBJParser_interleaved.js getDrawingInfo, filled from the mesh the caller
//     passes (the reference loader's triangles, tests/golden/gen_js_walk.py).
// Instrumentation: intersect_triangle is wrapped (the walk calls the global by
// name) to log the tested triangle ids in order, to record the id of the last
// accepted one and where the first accept came (the prefix an any-hit walk tests)
// -- the walk itself runs unmodified.
// usage: node gen_js_walk.js <reference js/bsp_tree/modules dir> <in.json> <out.json>
'use strict';
const fs = require('fs');
const vm = require('vm');
const crypto = require('crypto');
const [modDir, inPath, outPath] = process.argv.slice(2);
const inp = JSON.parse(fs.readFileSync(inPath, 'utf8'));

const sandbox = {
  console: { log() {}, error() {} },
  Math, Float32Array, Uint32Array, Map, Array, Object, parseInt, parseFloat, isNaN, isFinite,
  GPUBufferUsage: { COPY_DST: 0, STORAGE: 0, UNIFORM: 0 },
};
vm.createContext(sandbox);
vm.runInContext(`
function vec3(a, b, c) { return [a, b, c]; }
function vec4(v) { return [v[0], v[1], v[2], v.length > 3 ? v[3] : 1.0]; }
function subtract(u, v) { const r = []; for (let i = 0; i < u.length; ++i) r.push(u[i] - v[i]); return r; }
function cross(u, v) { return [u[1]*v[2] - u[2]*v[1], u[2]*v[0] - u[0]*v[2], u[0]*v[1] - u[1]*v[0]]; }
function dot(u, v) { let sum = 0.0; for (let i = 0; i < u.length; ++i) sum += u[i]*v[i]; return sum; }
function length(u) { return Math.sqrt(dot(u, u)); }
function normalize(u) { const len = length(u); const r = []; for (let i = 0; i < u.length; ++i) r.push(u[i]/len); return r; }
function flatten(vs) { const out = []; for (const v of vs) for (const x of v) out.push(x); return new Float32Array(out); }
`, sandbox);
vm.runInContext(fs.readFileSync(modDir + '/Aabb.js', 'utf8'), sandbox);
vm.runInContext(fs.readFileSync(modDir + '/BspTree_interleaved.js', 'utf8'), sandbox);

// g_drawingInfo in OBJParser_interleaved.js's layout
const nv = inp.pos.length / 3, nt = inp.idx.length / 4;
const attribs = new Float32Array(nv * 8);
for (let i = 0; i < nv; ++i) {
  attribs[i * 8] = inp.pos[i * 3]; attribs[i * 8 + 1] = inp.pos[i * 3 + 1]; attribs[i * 8 + 2] = inp.pos[i * 3 + 2];
  attribs[i * 8 + 3] = 1.0;
}
sandbox.g_drawingInfo = { attribs: attribs, colors: new Float32Array(nv * 4), indices: new Uint32Array(inp.idx) };
const device = { createBuffer: () => ({}), queue: { writeBuffer: () => {} } };
vm.runInContext('build_bsp_tree(g_drawingInfo, __device, {})', Object.assign(sandbox, { __device: device }));

vm.runInContext(`
var __log = [];
var __first = -1;   // tests up to and including the first accept (the any-hit walk's prefix)
const __intersect_triangle = intersect_triangle;
intersect_triangle = function (r, hit, idx) {
  __log.push(idx);
  const ok = __intersect_triangle(r, hit, idx);
  if (ok) hit.tri = idx;
  if (ok && __first < 0) __first = __log.length;
  return ok;
};
`, sandbox);

function fnv(ids) {   // FNV-1a 32 over the ids as little-endian u32
  let h = 0x811c9dc5;
  for (const v of ids) for (let b = 0; b < 4; ++b) { h ^= (v >>> (8 * b)) & 0xff; h = Math.imul(h, 0x01000193) >>> 0; }
  return h >>> 0;
}
const query = vm.runInContext(`(function (o, d, tmin, tmax, clip) {
  const ray = { origin: [o[0], o[1], o[2]], direction: [d[0], d[1], d[2]], tmin: tmin, tmax: tmax };
  const hit = { has_hit: false, dist: 0.0, tri: -1 };
  __log = [];
  __first = -1;
  let status;
  if (clip && !intersect_min_max(ray)) status = -1;
  else status = intersect_bsp_array(ray, hit) ? 1 : 0;
  return [status, hit.tri, hit.dist, ray.tmin, ray.tmax, __log.slice(), __first];
})`, sandbox);

const results = [];
for (const r of inp.rays) {
  const [st, tri, dist, t0, t1, log, first] = query(r[0], r[1], r[2], r[3], r[4]);
  const pre = first < 0 ? log : log.slice(0, first);
  results.push([st, tri, dist, t0, t1, log.length, fnv(log), pre.length, fnv(pre)]);
}
const tree = vm.runInContext('({ tree: bspTree, planes: bspPlanes, ids: treeIds })', sandbox);
const sha = crypto.createHash('sha256');
sha.update(Buffer.from(tree.tree.buffer)); sha.update(Buffer.from(tree.planes.buffer)); sha.update(Buffer.from(tree.ids.buffer));
fs.writeFileSync(outPath, JSON.stringify({ ntris: nt, nids: tree.ids.length, tree_sha256: sha.digest('hex'), results: results }));
