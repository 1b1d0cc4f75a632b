"""The data plane as Kubernetes runs it: one process per pod, each with the environment the nos
device plugin's ``Allocate`` gives its container (``procs``), running the demo client loop
(``client``)."""
