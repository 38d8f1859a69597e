// _lsr_autograd: two accessors of a leaf tensor's cached AccumulateGrad node, for the captured
// train steps (langsplat_amd/graph.py, langsplat_amd/pipeline.py).  Host code only, no GPU work.
//
// Why: autograd keeps one AccumulateGrad node per leaf tensor (the parameter) for as long as any
// autograd graph references it, and a node is bound to the stream that was current when it was
// created.  LangSplat's train loop keeps the previous iteration's render package and loss alive
// (/root/reference/train.py:92-108), so the parameters' nodes stay bound to the caller's stream.
// A HIP graph capture of the next step then reuses those nodes: the captured backward waits on the
// caller's (non-capturing) stream, torch warns "AccumulateGrad node's stream does not match", and
// this HIP runtime crashes at capture end.  Releasing the tensor's reference to the
// cached node before a capture makes the captured graph create its own node on the capture stream;
// the stale graph keeps its node (its backward, if ever run, still accumulates into .grad).
#include <Python.h>

#include <torch/csrc/autograd/function.h>
#include <torch/csrc/autograd/python_variable.h>
#include <torch/csrc/autograd/variable.h>

namespace {

bool unpack(PyObject* obj, at::Tensor& out)
{
    if (!THPVariable_Check(obj)) {
        PyErr_SetString(PyExc_TypeError, "_lsr_autograd: expected a torch.Tensor");
        return false;
    }
    out = THPVariable_Unpack(obj);
    return true;
}

// accumulator_stream(t) -> None if t has no live AccumulateGrad node, else (device_index, stream_id)
// of the stream the node was created on (compare torch.cuda.Stream.device_index / .stream_id)
PyObject* accumulator_stream(PyObject*, PyObject* arg)
{
    at::Tensor t;
    if (!unpack(arg, t)) return nullptr;
    auto node = torch::autograd::impl::try_get_grad_accumulator(t);
    if (!node) Py_RETURN_NONE;
    auto st = node->stream();
    if (!st.has_value()) Py_RETURN_NONE;
    return Py_BuildValue("(iL)", (int)st->device_index(), (long long)st->id());
}

// release_accumulator(t) -> True if t had a live AccumulateGrad node; the tensor forgets it (the next
// graph that uses t creates a fresh node on the then-current stream)
PyObject* release_accumulator(PyObject*, PyObject* arg)
{
    at::Tensor t;
    if (!unpack(arg, t)) return nullptr;
    if (!t.requires_grad() || !t.is_leaf()) {
        PyErr_SetString(PyExc_ValueError, "_lsr_autograd.release_accumulator: a leaf tensor that requires grad");
        return nullptr;
    }
    auto node = torch::autograd::impl::try_get_grad_accumulator(t);
    if (!node) Py_RETURN_FALSE;
    torch::autograd::impl::set_grad_accumulator(t, std::weak_ptr<torch::autograd::Node>());
    Py_RETURN_TRUE;
}

PyMethodDef methods[] = {
    {"accumulator_stream", accumulator_stream, METH_O,
     "(device_index, stream_id) of a leaf's live AccumulateGrad node, or None"},
    {"release_accumulator", release_accumulator, METH_O,
     "drop a leaf's reference to its cached AccumulateGrad node; True if it had one"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_lsr_autograd", nullptr, -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__lsr_autograd() { return PyModule_Create(&module); }
