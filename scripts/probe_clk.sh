ls /sys/class/drm/ | head -20
for c in /sys/class/drm/card*/device; do echo "$c: $(cat $c/uevent 2>/dev/null | grep PCI_SLOT_NAME)"; head -3 $c/pp_dpm_sclk 2>&1 | tr '\n' ' '; echo; ls -la $c/gpu_metrics 2>&1 | head -1; done 2>&1 | head -40
python3 -c "
import torch
p=torch.cuda.get_device_properties(0)
print([a for a in dir(p) if not a.startswith('_')])
print(getattr(p,'pci_bus_id',None), getattr(p,'pci_device_id',None), getattr(p,'pci_domain_id',None))
"
which amd-smi; python3 -c "import amdsmi; print('amdsmi ok')" 2>&1 | tail -1
