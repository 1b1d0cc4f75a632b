"""A node's kubelet as far as the partition agent and its device plugins can tell — for running the
real agent binary outside a cluster (``cmd/devcluster.py``, ``tests/test_e2e_processes.py``).

* the **Registration** endpoint (``<dir>/kubelet.sock``) the nos device plugins register with;
* one **ListAndWatch** reader per registered resource, holding the plugin's latest device list
  (re-opened when a plugin re-registers on a new endpoint);
* **admission**: a bound pod gets a healthy, unallocated device of its resource through the
  plugin's own ``Allocate`` over gRPC, or fails as ``UnexpectedAdmissionError``, as kubelet does;
* the **PodResources** endpoint (``<dir>/../pod-resources.sock``) reporting the devices of running
  pods, which the agent reads to know what is in use.

Node status (allocatable) is the agent's to publish (``publishAllocatable``); this kubelet only
moves pods to ``Running`` / ``Failed`` / ``Succeeded``.
"""
from __future__ import annotations

import os
import threading
from typing import Any, Dict, List, Optional, Tuple

import grpc

from ..device.podresources import PodResourcesServer
from ..device.protos import dp
from ..deviceplugin.server import RegistrationServer
from ..kube import objects as ko


class FakeKubelet:
    def __init__(self, root: str, client: Any, node: str):
        self.root = root
        self.dir = os.path.join(root, "device-plugins")
        os.makedirs(self.dir, exist_ok=True)
        self.client = client
        self.node = node
        self.reg = RegistrationServer(os.path.join(self.dir, "kubelet.sock")).start()
        self.devices: Dict[str, List[Tuple[str, str]]] = {}      # resource -> [(id, health)]
        self.readers: Dict[str, Tuple[int, threading.Thread]] = {}  # resource -> (registration #, reader)
        self.used: Dict[Tuple[str, str], Tuple[str, str]] = {}   # (ns, pod) -> (resource, id)
        self.admission_failures: List[Tuple[Tuple[str, str], str]] = []
        self.allocations: Dict[Tuple[str, str], List[str]] = {}  # (ns, pod) -> host device paths
        self.envs: Dict[Tuple[str, str], Dict[str, str]] = {}     # (ns, pod) -> env Allocate injected
        self.lock = threading.Lock()
        self._published: set = set()
        self.podres_socket = os.path.join(root, "pod-resources.sock")
        self.podres = PodResourcesServer(self.podres_socket, self._used, self._alloc).start()

    # -- PodResources --------------------------------------------------------------------
    def _used(self):
        with self.lock:
            return [(p, ns, [(r, [i])]) for (ns, p), (r, i) in self.used.items()]

    def _alloc(self):
        with self.lock:
            return [(r, [i for i, _ in ds]) for r, ds in self.devices.items()]

    # -- device plugins ------------------------------------------------------------------
    def _read(self, resource: str, endpoint: str) -> None:
        ch = grpc.insecure_channel("unix://" + os.path.join(self.dir, endpoint))
        law = ch.unary_stream(f"/{dp.SERVICE}/ListAndWatch", request_serializer=dp.Empty.SerializeToString,
                              response_deserializer=dp.ListAndWatchResponse.FromString)
        try:
            for resp in law(dp.Empty()):
                with self.lock:
                    self.devices[resource] = [(x.ID, x.health) for x in resp.devices]
        except grpc.RpcError:
            pass
        finally:
            ch.close()
            # the plugin went away (restart, crash): its devices are gone until it registers again,
            # as kubelet drops a plugin's devices when its endpoint closes
            with self.lock:
                self.devices.pop(resource, None)

    def sync(self) -> None:
        """Open a ListAndWatch stream for every *new registration* (a resource registered for the
        first time, or registered again), and publish the node's allocatable (healthy devices) and
        capacity (all devices), as kubelet's node-status sync does.  A stream that ended is not
        reopened on its own: kubelet drops the endpoint and waits for the plugin to register
        again, so a plugin whose stream dies must notice and re-register."""
        latest: Dict[str, Tuple[int, str]] = {}
        for k, r in enumerate(self.reg.registered):
            latest[r.resource_name] = (k, r.endpoint)
        for res, (k, ep) in latest.items():
            cur = self.readers.get(res)
            if cur is None or cur[0] != k:
                t = threading.Thread(target=self._read, args=(res, ep), daemon=True, name=f"law-{res}")
                t.start()
                self.readers[res] = (k, t)
        self._publish()

    def endpoint(self, resource: str) -> str:
        k, _ = self.readers[resource]
        return self.reg.registered[k].endpoint

    def _publish(self) -> None:
        with self.lock:
            alloc = {r: str(sum(1 for _, h in ds if h == dp.HEALTHY)) for r, ds in self.devices.items()}
            cap = {r: str(len(ds)) for r, ds in self.devices.items()}
        for r in self._published - set(alloc):   # a resource whose plugin is gone counts 0
            alloc[r] = cap[r] = "0"
        self._published |= set(alloc)
        if not alloc:
            return
        st = (self.client.get("Node", self.node).get("status") or {})
        if all(st.get("allocatable", {}).get(r) == v for r, v in alloc.items()) and \
                all(st.get("capacity", {}).get(r) == v for r, v in cap.items()):
            return
        self.client.patch("Node", self.node, {"status": {"allocatable": alloc, "capacity": cap}})

    def healthy(self, resource: str) -> List[str]:
        with self.lock:
            return [i for i, h in self.devices.get(resource, []) if h == dp.HEALTHY]

    # -- pods ----------------------------------------------------------------------------
    def admit(self, pod: Dict[str, Any], node: str = "") -> Optional[str]:
        """kubelet admission of a pod just bound here (``KubeScheduler``'s ``on_bind``). Returns
        the device id, or None after marking the pod Failed."""
        reqs = {}
        for c in pod["spec"].get("containers", []):
            reqs.update((c.get("resources") or {}).get("requests") or {})
            reqs.update((c.get("resources") or {}).get("limits") or {})
        res = next((k for k in reqs if k.startswith("amd.com/") and k != "amd.com/gpu"), None)
        key = (ko.namespace(pod), ko.name(pod))
        if res is None:
            self.client.patch("Pod", key[1], {"status": {"phase": "Running"}}, key[0])
            return None
        with self.lock:
            taken = {i for _, i in self.used.values()}
            free = [i for i, h in self.devices.get(res, []) if h == dp.HEALTHY and i not in taken]
        try:
            if not free:
                raise RuntimeError(f"no healthy {res} device")
            ch = grpc.insecure_channel("unix://" + os.path.join(self.dir, self.endpoint(res)))
            req = dp.AllocateRequest()
            req.container_requests.add(devicesIDs=[free[0]])
            try:
                resp = ch.unary_unary(f"/{dp.SERVICE}/Allocate", request_serializer=dp.AllocateRequest.SerializeToString,
                                      response_deserializer=dp.AllocateResponse.FromString)(req, timeout=5)
            finally:
                ch.close()
            if not resp.container_responses or not resp.container_responses[0].devices:
                raise RuntimeError("Allocate returned no device")
        except Exception as e:  # noqa: BLE001 - an admission failure is a pod outcome
            self.admission_failures.append((key, str(e)))
            self.client.patch("Pod", key[1], {"status": {"phase": "Failed", "reason": "UnexpectedAdmissionError",
                                                         "message": str(e)}}, key[0])
            return None
        with self.lock:
            self.used[key] = (res, free[0])
            self.allocations[key] = [d.host_path for d in resp.container_responses[0].devices]
            self.envs[key] = dict(resp.container_responses[0].envs)
        self.client.patch("Pod", key[1], {"status": {"phase": "Running"}}, key[0])
        return free[0]

    def finish(self, namespace: str, name: str, delete: bool = True) -> None:
        """The pod's containers exit: its device is released (and the pod deleted)."""
        with self.lock:
            self.used.pop((namespace, name), None)
        self.client.patch("Pod", name, {"status": {"phase": "Succeeded"}}, namespace)
        if delete:
            self.client.delete("Pod", name, namespace)

    def stop(self) -> None:
        self.reg.stop()
        self.podres.stop()
