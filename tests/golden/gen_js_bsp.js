// Generates BSP golden fixtures by RUNNING the reference's own instructor
// JavaScript BSP builder (js/bsp_tree/BspRunner.js in the reference checkout)
// under node.  Nothing from the reference is copied: the script is read from
// the path given on the command line and evaluated in a vm sandbox with stubs
// for the browser APIs it touches (fetch, XMLHttpRequest, console).
// usage: node gen_js_bsp.js <BspRunner.js> <model.obj> <out.json>
'use strict';
const fs = require('fs');
const vm = require('vm');
const [runner, objPath, outPath] = process.argv.slice(2);
const src = fs.readFileSync(runner, 'utf8');
const sandbox = {
  console: { log() {}, error() {} },
  fetch: () => ({ then: () => ({ then: () => ({ catch: () => {} }) }) }),
  XMLHttpRequest: function () {
    this.open = () => {}; this.send = () => { this.readyState = 4; this.status = 404;
      if (this.onreadystatechange) this.onreadystatechange(); };
  },
  Math, Float32Array, Uint32Array, Map, Array, Object, parseInt, parseFloat, isNaN,
};
vm.createContext(sandbox);
vm.runInContext(src, sandbox);
const text = fs.readFileSync(objPath, 'utf8');
const out = vm.runInContext(`(function(text){
  const doc = new OBJDoc("model.obj");
  doc.parse(text, 1.0, false);
  const di = doc.getDrawingInfo();
  build_bsp_tree(di);
  const nodes = [];
  for (let i = 0; i < bspPlanes.length; i++) {
    const a = bspTree[i*4], b = bspTree[i*4+1], c = bspTree[i*4+2], d = bspTree[i*4+3];
    if (a || b || c || d || bspPlanes[i]) nodes.push([i, a, b, c, d, bspPlanes[i]]);
  }
  return { ntris: di.indices.length / 4, max_level: max_level, max_objects: max_objects,
           nnodes: bspPlanes.length, nodes: nodes, tree_ids: Array.from(treeIds),
           bbox: [root.bbox.min[0], root.bbox.min[1], root.bbox.min[2], root.bbox.max[0], root.bbox.max[1], root.bbox.max[2]] };
})`, sandbox)(text);
fs.writeFileSync(outPath, JSON.stringify(out));
